# Relay cap lines / 64 (this build) vs lines / 512 below 64 lines and
# lines / 256 above (abtest/base.so): relay tests, then chunk-form and
# descriptor shapes, one library per process.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cd2.log 2>&1
export SWEEP_ONLY="4096:65536,4096:73728,4096:81920,4096:98304,4096:139264,4096:147456,4096:163840,8192:98304,8192:106496,16384:98304,16384:106496,2048:81920,2048:139264,32768:98304,32768:106496,32768:1048577"
for r in 1 2; do
  step new 200 python -u tools/shape_sweep.py >> gpurun_out/cd2_new.log 2>&1
  CIRUELA_AMD_LIB=abtest/base.so step old 200 python -u tools/shape_sweep.py >> gpurun_out/cd2_old.log 2>&1
  SWEEP_DESC=1 step dnew 200 python -u tools/shape_sweep.py >> gpurun_out/cd2_dnew.log 2>&1
  SWEEP_DESC=1 CIRUELA_AMD_LIB=abtest/base.so step dold 200 python -u tools/shape_sweep.py >> gpurun_out/cd2_dold.log 2>&1
done
