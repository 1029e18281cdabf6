# Relay cap lines / 32 vs lines / 64 (default) at 5/8 of a lane wave of
# 32-line chains and 1/2 - 5/8 of 16-line ones, files and descriptors.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="4096:102400,4096:106496,4096:172032,2048:90112,2048:98304,2048:106496,2048:163840,2048:65536"
for r in 1 2; do
  step c64 200 python -u tools/shape_sweep.py >> gpurun_out/cd3_64.log 2>&1
  CIR_RELAY_CAPDIV=32 step c32 200 python -u tools/shape_sweep.py >> gpurun_out/cd3_32.log 2>&1
done
