# k = 1 quad-regime relay: segment floor 32 (default) vs 64 / 128 lines.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:16384,32768:16385,32768:17408,32768:18432,32768:20480,32768:22528,32768:24576,262144:16385,262144:20480,16384:20480,1048576:20480"
for r in 1 2; do
  step s32 200 python -u tools/shape_sweep.py >> gpurun_out/qseg1_32.log 2>&1
  CIR_RELAY_QSEG1=64 step s64 200 python -u tools/shape_sweep.py >> gpurun_out/qseg1_64.log 2>&1
  CIR_RELAY_QSEG1=128 step s128 200 python -u tools/shape_sweep.py >> gpurun_out/qseg1_128.log 2>&1
done
