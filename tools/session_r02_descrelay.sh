# Descriptor relay: GPU tests (relay + descriptor paths + chunk relay), the
# descriptor shapes prev (no descriptor relay) vs cur, config 3 / quad A/B.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
CIRUELA_AMD_LIB=abtest/cur.so step tests 900 python -u -m pytest tests/test_gpu_parity.py -x -v -k "relay or desc or golden or random or verify or host_blocks or hash_file or scan or memory" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dr.log 2>&1
CIRUELA_AMD_LIB=abtest/cur.so step tests_full 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "config3" --timeout 300 --timeout-method thread -p no:cacheprovider >> gpurun_out/pytest_dr.log 2>&1
export SWEEP_DESC=1 SWEEP_ONLY="32768:65536,32768:65537,32768:66560,32768:73728,32768:98304,32768:106496,32768:131072,32768:131073,32768:147456,262144:65536,262144:65537,262144:73728,4096:65536,4096:65537,4096:69632,4096:131073,16384:65537"
for r in 1 2; do
  for lib in prev cur; do
    CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 300 python -u tools/shape_sweep.py >> gpurun_out/dr_$lib.log 2>&1
  done
done
step ab 900 bash tools/ab_proc.sh 2 abtest/prev.so abtest/cur.so > gpurun_out/ab_dr.log 2>&1
