# Quad-regime relay: new defaults (relay first, 8-line segments, >= 64/32 lines)
# against the previous ones (base first, 16-line segments, >= 128 lines).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qs2.log 2>&1
export SWEEP_ONLY="32768:16384,32768:16385,32768:20480,32768:32768,32768:32769,32768:33792,32768:36864,32768:49152,32768:49153,262144:16385,262144:32769,262144:49153,1048576:32769,1048576:49153,8192:32769,16384:32769,4096:32768,4096:32769"
for r in 1 2; do
  CIR_RELAY=0 step off 200 python -u tools/shape_sweep.py >> gpurun_out/qs2_off.log 2>&1
  step new 200 python -u tools/shape_sweep.py >> gpurun_out/qs2_new.log 2>&1
  CIR_RELAY_QLINES=128 CIR_RELAY_QSEG=16 CIR_RELAY_QFIRST=0 step old 200 python -u tools/shape_sweep.py >> gpurun_out/qs2_old.log 2>&1
done
