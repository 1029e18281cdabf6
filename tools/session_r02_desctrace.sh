# Kernel trace of descriptor batches of equal long blocks.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_DESC=1 SWEEP_STEPS=2 SWEEP_ONLY="262144:65536,262144:16384,262144:32768,1048576:16384,1048576:20000"
step trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/desc_trace -o run -- python3 tools/shape_sweep.py > gpurun_out/desc_trace.log 2>&1
