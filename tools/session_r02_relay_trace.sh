# Relay timeline: kernel trace of a few relayed shapes (one process).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="4096:65537,32768:65537,32768:32769,32768:16385" SWEEP_STEPS=3
step trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/relay_trace -o run -- python3 tools/shape_sweep.py > gpurun_out/relay_trace.log 2>&1
