# Prefetching lane part at 4 waves/SIMD (10 VGPRs spilled outside the
# compression bodies) vs 3 (no spills) vs the previous lane part.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_DESC=1 SWEEP_ONLY="32768:49153,32768:65536,32768:98304,32768:131072,32768:262144,32768:1048576,262144:65536,4096:65536,4096:1048576,4096:4194304,65536:65536,131072:100000"
for r in 1 2; do
  for lib in prev cur4 cur3; do
    CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 300 python -u tools/shape_sweep.py >> gpurun_out/lpf2_$lib.log 2>&1
  done
done
CIRUELA_AMD_LIB=abtest/cur4.so step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "desc or golden or random or verify or host_blocks" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lpf2.log 2>&1
