# Quad-regime relay for short chains (4 KiB / 8 KiB blocks): variants.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="4096:16384,4096:16385,4096:32768,4096:32769,8192:16384,8192:16385,8192:32768,8192:32769,16384:32768,16384:32769"
export CIR_RELAY_QLINES=16
for r in 1 2; do
  CIR_RELAY=0 step off 120 python -u tools/shape_sweep.py >> gpurun_out/qs_off.log 2>&1
  step pad 120 python -u tools/shape_sweep.py >> gpurun_out/qs_pad.log 2>&1
  CIR_RELAY_QPAD=0 CIR_RELAY_QFIRST=1 step nopad_first 120 python -u tools/shape_sweep.py >> gpurun_out/qs_nopad_first.log 2>&1
  CIR_RELAY_QFIRST=1 CIR_RELAY_QSEG=8 step pad_first8 120 python -u tools/shape_sweep.py >> gpurun_out/qs_pad_first8.log 2>&1
done
