# Small descriptor batches with both parts on one stream (no fork/join to
# the quad-part stream when no relay runs) vs the previous build
# (abtest/base.so): desc tests, then the sweep, one library per process.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "desc or blocks or relay or concurrent" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_serial.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:16384,8192:24576,32768:32768,1048576:16384,4096:16384,32768:24576,32768:45056,1048576:20000,65536:8192,32768:1024"
for r in 1 2; do
  step new 200 python -u tools/shape_sweep.py >> gpurun_out/serial_new.log 2>&1
  CIRUELA_AMD_LIB=abtest/base.so step old 200 python -u tools/shape_sweep.py >> gpurun_out/serial_old.log 2>&1
done
