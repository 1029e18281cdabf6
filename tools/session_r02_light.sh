# Relay hand-off: fences (light0) vs agent-scope state loads/stores (light1).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
CIRUELA_AMD_LIB=abtest/light1.so step tests 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay or desc" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_light.log 2>&1
export SWEEP_ONLY="32768:16384,32768:16385,262144:16384,262144:16385,32768:32769,4096:65536,4096:65537,32768:65537,262144:65537,1048576:32769"
for r in 1 2; do
  for lib in light0 light1; do
    CIRUELA_AMD_LIB=abtest/$lib.so step c_$lib 300 python -u tools/shape_sweep.py >> gpurun_out/l_c_$lib.log 2>&1
    SWEEP_DESC=1 SWEEP_ONLY="32768:16384,32768:16385,1048576:20000,32768:65537,4096:65537" CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 300 python -u tools/shape_sweep.py >> gpurun_out/l_d_$lib.log 2>&1
  done
done
