# Segment waves per relay (CIR_RELAY_SEGS; default one per SIMD) vs half
# and twice that.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:65537,32768:73728,32768:98304,32768:106496,4096:73728,4096:139264,32768:16385,32768:24576,262144:32769,32768:1114113"
for r in 1 2; do
  step def 200 python -u tools/shape_sweep.py >> gpurun_out/sg_def.log 2>&1
  CIR_RELAY_SEGS=512 step s512 200 python -u tools/shape_sweep.py >> gpurun_out/sg_512.log 2>&1
  CIR_RELAY_SEGS=2048 step s2048 200 python -u tools/shape_sweep.py >> gpurun_out/sg_2048.log 2>&1
done
