# Relay tests after the short-chain cap, and the 4 KiB shapes around it.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cap.log 2>&1
export SWEEP_ONLY="4096:65536,4096:65537,4096:66560,4096:69632,4096:69633,4096:73728,4096:131072,4096:131073,4096:135168,4096:139264,8192:65537,8192:81920"
for r in 1 2; do
  CIR_RELAY=0 step off 200 python -u tools/shape_sweep.py >> gpurun_out/cap_off.log 2>&1
  step on 200 python -u tools/shape_sweep.py >> gpurun_out/cap_on.log 2>&1
done
