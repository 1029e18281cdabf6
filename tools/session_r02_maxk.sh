# Relays past 16 lane waves per SIMD (CIR_RELAY_MAXK = 16 default vs 32).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:1114112,32768:1114113,32768:1130496,32768:1310720,32768:1310721,4096:1114113,4096:1310721"
export SWEEP_STEPS=6
for r in 1 2; do
  step k16 300 python -u tools/shape_sweep.py >> gpurun_out/mk_16.log 2>&1
  CIR_RELAY_MAXK=32 step k32 300 python -u tools/shape_sweep.py >> gpurun_out/mk_32.log 2>&1
  SWEEP_DESC=1 step d16 300 python -u tools/shape_sweep.py >> gpurun_out/mk_d16.log 2>&1
  SWEEP_DESC=1 CIR_RELAY_MAXK=32 step d32 300 python -u tools/shape_sweep.py >> gpurun_out/mk_d32.log 2>&1
done
