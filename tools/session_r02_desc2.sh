# Descriptor batches: prefetching lane part + no quad part when the long
# chains overflow it (cur) vs HEAD before (prev); config 3 and quad workloads.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
CIRUELA_AMD_LIB=abtest/cur.so step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "desc or golden or random or verify or host_blocks or hash_file or scan or memory" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_desc2.log 2>&1
CIRUELA_AMD_LIB=abtest/cur.so step tests_full 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "config3" --timeout 300 --timeout-method thread -p no:cacheprovider >> gpurun_out/pytest_desc2.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:49153,32768:65536,32768:65537,32768:98304,32768:131072,262144:49153,262144:65536,262144:65537,131072:100000,131072:16384,131072:20000,1048576:16384,1048576:20000,4096:65536,4096:1048576,65536:65536"
for r in 1 2; do
  for lib in prev cur; do
    CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 300 python -u tools/shape_sweep.py >> gpurun_out/desc2_$lib.log 2>&1
  done
done
step ab 900 bash tools/ab_proc.sh 2 abtest/prev.so abtest/cur.so > gpurun_out/ab_desc2.log 2>&1
