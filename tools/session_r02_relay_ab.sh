# Relay A/B on a few shapes (relay off / on), plus the relay tests.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "relay" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_relay.log 2>&1
export SWEEP_ONLY="32768:16384,32768:16385,32768:20480,262144:16384,262144:16385,4096:65536,4096:65537,32768:65536,32768:65537,32768:32768,32768:32769,262144:65537,1048576:32769"
CIR_RELAY=0 step sweep_off 300 python -u tools/shape_sweep.py > gpurun_out/sweep_off.log 2>&1
step sweep_on 300 python -u tools/shape_sweep.py > gpurun_out/sweep_on.log 2>&1
