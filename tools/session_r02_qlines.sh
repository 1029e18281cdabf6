# Quad-regime relay of short chains after the fence-free hand-off: the
# shortest relayed chain (CIR_RELAY_QLINES; default 64 at k = 1, 32 above).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="4096:16384,4096:16385,4096:16400,4096:17408,4096:20480,4096:32768,4096:32769,4096:33792,4096:36864,2048:32769,2048:36864,4096:106496,4096:114688"
for r in 1 2; do
  step def 200 python -u tools/shape_sweep.py >> gpurun_out/ql_def.log 2>&1
  CIR_RELAY_QLINES=32 step q32 200 python -u tools/shape_sweep.py >> gpurun_out/ql_32.log 2>&1
  CIR_RELAY_QLINES=16 CIR_RELAY_CAPDIV=32 step q16 200 python -u tools/shape_sweep.py >> gpurun_out/ql_16.log 2>&1
done
