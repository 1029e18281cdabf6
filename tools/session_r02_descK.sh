# Descriptor relay beyond k = 2 lane waves per SIMD (lane part padded to two
# waves per SIMD beside it): shapes prev (k <= 2) vs cur (k <= 16), tests.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_DESC=1 SWEEP_ONLY="32768:196608,32768:196609,32768:212992,32768:262144,32768:262145,32768:524288,32768:524289,32768:1048576,32768:1048577,32768:1064960,4096:262145,4096:1048577"
for r in 1 2; do
  for lib in prev cur; do
    CIRUELA_AMD_LIB=abtest/$lib.so step d_$lib 400 python -u tools/shape_sweep.py >> gpurun_out/dk_$lib.log 2>&1
  done
done
