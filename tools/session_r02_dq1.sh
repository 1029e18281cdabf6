# Descriptor batch of exactly one quad wave per SIMD (32 KiB x 16384) vs the
# chunk form: kernel trace of both (where the desc path's extra time goes).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:16384,8192:24576" SWEEP_STEPS=20
export SWEEP_DESC=1
step desc 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/dq1_desc -o run -- python3 -u tools/shape_sweep.py > gpurun_out/dq1_desc.log 2>&1
export SWEEP_DESC=0
step chunk 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/dq1_chunk -o run -- python3 -u tools/shape_sweep.py > gpurun_out/dq1_chunk.log 2>&1
