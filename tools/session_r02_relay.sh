# Relay session: the relay GPU tests, then the shape sweep with and without
# the relay (and with the quad-regime floor at k = 1).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "relay" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_relay.log 2>&1
CIR_RELAY=0 step sweep_off 400 python -u tools/shape_sweep.py > gpurun_out/sweep_off.log 2>&1
step sweep_on 400 python -u tools/shape_sweep.py > gpurun_out/sweep_on.log 2>&1
SWEEP_ONLY="32768:16384,32768:16385,32768:20480,4096:16384,4096:16385,262144:16384,262144:16385" step sweep_q1 200 python -u tools/shape_sweep.py > gpurun_out/sweep_q1.log 2>&1
