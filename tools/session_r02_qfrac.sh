# Quad-regime relay: how large a fraction of a quad wave per SIMD of extra
# chains still pays (CIR_RELAY_QFRAC = d: relay when extra <= quad_slots / d).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:16384,32768:20480,32768:24576,32768:28672,32768:32768,32768:36864,32768:40960,32768:45056,262144:24576,262144:40960,1048576:24576,16384:24576,65536:24576,65536:40960"
for r in 1 2; do
  step d4 200 python -u tools/shape_sweep.py >> gpurun_out/qf_d4.log 2>&1
  CIR_RELAY_QFRAC=2 step d2 200 python -u tools/shape_sweep.py >> gpurun_out/qf_d2.log 2>&1
  CIR_RELAY_QFRAC=1 step d1 200 python -u tools/shape_sweep.py >> gpurun_out/qf_d1.log 2>&1
done
