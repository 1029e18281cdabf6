# Descriptor relay gate A/B: gate on (default) / off, cap 1/2 / 5/8.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay or desc" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gate.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:65536,32768:65537,32768:73728,32768:81920,32768:98304,32768:106496,32768:131073,32768:196609,4096:65537,262144:65537"
for r in 1 2; do
  CIR_RELAY_GATE=0 step nogate 300 python -u tools/shape_sweep.py >> gpurun_out/g_nogate.log 2>&1
  step gate 300 python -u tools/shape_sweep.py >> gpurun_out/g_gate.log 2>&1
  CIR_RELAY_DCAP8=5 step gate58 300 python -u tools/shape_sweep.py >> gpurun_out/g_gate58.log 2>&1
done
