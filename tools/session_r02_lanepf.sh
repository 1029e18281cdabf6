# Lane part with line prefetch (k_lane_rest, 3 waves/SIMD) vs without (4):
# descriptor shapes, config 3 and the quad workloads, GPU tests of the path.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "desc or golden or random or verify or host_blocks or hash_file or scan" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lpf.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:49153,32768:65536,32768:65537,32768:98304,32768:131072,262144:65536,262144:49153,4096:65536,4096:1048576,65536:65536,1048576:20000,131072:100000"
for r in 1 2; do
  CIRUELA_AMD_LIB=abtest/prev.so step d_prev 300 python -u tools/shape_sweep.py >> gpurun_out/lpf_prev.log 2>&1
  CIRUELA_AMD_LIB=abtest/cur.so step d_cur 300 python -u tools/shape_sweep.py >> gpurun_out/lpf_cur.log 2>&1
done
step ab 900 bash tools/ab_proc.sh 2 abtest/prev.so abtest/cur.so > gpurun_out/ab_lpf.log 2>&1
