# Quad-regime descriptor relay on qs (base on the lane stream): tests, shapes.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay or desc or golden or random or concurrent or quad" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qd2.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:16384,32768:16385,32768:20000,32768:32768,32768:32769,65536:16385,1048576:16384,1048576:20000,8192:32769,32768:65537"
for r in 1 2; do
  CIR_RELAY=0 step off 300 python -u tools/shape_sweep.py >> gpurun_out/qd2_off.log 2>&1
  step on 300 python -u tools/shape_sweep.py >> gpurun_out/qd2_on.log 2>&1
done
