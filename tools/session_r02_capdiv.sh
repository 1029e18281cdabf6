# Lane-regime relay cap for short chains: lines / d of a lane wave per SIMD
# (CIR_RELAY_CAPDIV = d; default 512 below 64 lines, 256 above).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="4096:65536,4096:69632,4096:73728,4096:81920,4096:98304,4096:131072,4096:135168,4096:139264,4096:147456,4096:163840,4096:196608,4096:204800,4096:212992,8192:73728,8192:81920,8192:98304,8192:139264,8192:147456,2048:73728,2048:139264"
for r in 1 2; do
  step d0 200 python -u tools/shape_sweep.py >> gpurun_out/cd_def.log 2>&1
  CIR_RELAY_CAPDIV=256 step d256 200 python -u tools/shape_sweep.py >> gpurun_out/cd_256.log 2>&1
  CIR_RELAY_CAPDIV=128 step d128 200 python -u tools/shape_sweep.py >> gpurun_out/cd_128.log 2>&1
  CIR_RELAY_CAPDIV=64 step d64 200 python -u tools/shape_sweep.py >> gpurun_out/cd_64.log 2>&1
done
