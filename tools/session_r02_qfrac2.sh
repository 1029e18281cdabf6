# Half-wave quad-regime relay as the default: relay tests, then chunk-form
# and descriptor A/B against the previous 1/4 limit.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qf2.log 2>&1
export SWEEP_ONLY="32768:16384,32768:20480,32768:22528,32768:24576,32768:32768,32768:40960,32768:45056,262144:24576,1048576:24576,1048576:20000,16384:24576,8192:24576,65536:40960"
for r in 1 2; do
  step new 200 python -u tools/shape_sweep.py >> gpurun_out/qf2_new.log 2>&1
  CIR_RELAY_QFRAC=4 step old 200 python -u tools/shape_sweep.py >> gpurun_out/qf2_old.log 2>&1
  SWEEP_DESC=1 step dnew 200 python -u tools/shape_sweep.py >> gpurun_out/qf2_dnew.log 2>&1
  SWEEP_DESC=1 CIR_RELAY_DQFRAC=4 step dold 200 python -u tools/shape_sweep.py >> gpurun_out/qf2_dold.log 2>&1
done
