# Lane-regime relay cap past 5/8 of a lane wave per SIMD: files
# (CIR_RELAY_CAP8) and descriptors (CIR_RELAY_DCAP8), eighths of a wave.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_ONLY="32768:106496,32768:114688,32768:122880,32768:180224,32768:188416,4096:114688,4096:122880,262144:114688,16384:114688"
for r in 1 2; do
  step c5 200 python -u tools/shape_sweep.py >> gpurun_out/c8_5.log 2>&1
  CIR_RELAY_CAP8=6 step c6 200 python -u tools/shape_sweep.py >> gpurun_out/c8_6.log 2>&1
  CIR_RELAY_CAP8=7 step c7 200 python -u tools/shape_sweep.py >> gpurun_out/c8_7.log 2>&1
  SWEEP_DESC=1 step d5 200 python -u tools/shape_sweep.py >> gpurun_out/c8_d5.log 2>&1
  SWEEP_DESC=1 CIR_RELAY_DCAP8=6 step d6 200 python -u tools/shape_sweep.py >> gpurun_out/c8_d6.log 2>&1
  SWEEP_DESC=1 CIR_RELAY_DCAP8=7 step d7 200 python -u tools/shape_sweep.py >> gpurun_out/c8_d7.log 2>&1
done
