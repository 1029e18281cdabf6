# Quad loop A/B: the next line's LDS reads all ahead of the compression
# (rdi0) vs spread over its G steps (rdi1); one library per process.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "quad or relay or golden or hash_bytes or desc or scan_long or random" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rdi.log 2>&1
for lib in rdi0 rdi1; do
  CIRUELA_AMD_LIB=abtest/$lib.so step probe_$lib 200 python -u tools/quad_probe.py > gpurun_out/quad_probe_$lib.log 2>&1
done
step ab 900 bash tools/ab_proc.sh 3 abtest/rdi0.so abtest/rdi1.so > gpurun_out/ab_rdi.log 2>&1
