# Quad-regime descriptor relay: GPU tests, descriptor shapes prev vs cur,
# config 3 and the quad workloads.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
CIRUELA_AMD_LIB=abtest/cur.so step tests 900 python -u -m pytest tests/test_gpu_parity.py -x -v -k "relay or desc or golden or random or verify or host_blocks or hash_file or scan or memory or quad" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qd.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:16384,32768:16385,32768:20000,32768:32768,32768:32769,32768:36864,65536:16384,65536:16385,1048576:16384,1048576:16385,1048576:20000,4096:32768,4096:32769,8192:32769,32768:49152,32768:49153"
for r in 1 2; do
  for lib in prev cur; do
    CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 400 python -u tools/shape_sweep.py >> gpurun_out/qd_$lib.log 2>&1
  done
done
step ab 900 bash tools/ab_proc.sh 2 abtest/prev.so abtest/cur.so > gpurun_out/ab_qd.log 2>&1
