# Relay with the segment's first lines loaded before the wait: relay tests,
# relay shapes (prev build vs current, k = 1 quad segments 32 vs 16), and the
# quad-mode workloads of the split quad_fast (prev vs current).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "relay or quad or hash_bytes or scan_long" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pf.log 2>&1
export SWEEP_ONLY="32768:16384,32768:16385,32768:20480,262144:16384,262144:16385,4096:65536,4096:65537,32768:65536,32768:65537,32768:32768,32768:32769,262144:65537,1048576:32769,32768:131072,32768:131073"
for r in 1 2; do
  CIRUELA_AMD_LIB=abtest/prev.so step sw_prev 300 python -u tools/shape_sweep.py >> gpurun_out/sw_prev.log 2>&1
  CIRUELA_AMD_LIB=abtest/cur.so step sw_cur 300 python -u tools/shape_sweep.py >> gpurun_out/sw_cur.log 2>&1
  CIR_RELAY_QSEG1=16 CIRUELA_AMD_LIB=abtest/cur.so step sw_cur16 300 python -u tools/shape_sweep.py >> gpurun_out/sw_cur16.log 2>&1
done
step ab 900 bash tools/ab_proc.sh 2 abtest/prev.so abtest/cur.so > gpurun_out/ab_pf.log 2>&1
