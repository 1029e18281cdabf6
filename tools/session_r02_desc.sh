# Descriptor batches of equal blocks around whole waves per SIMD.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
export SWEEP_DESC=1 SWEEP_ONLY="32768:16384,32768:16385,32768:32768,32768:32769,32768:49152,32768:49153,32768:65536,32768:65537,32768:73728,32768:98304,32768:131072,32768:131073,32768:196608,32768:196609,262144:65536,262144:65537,4096:65536,4096:65537,4096:1048576,4096:1048577"
step desc 300 python -u tools/shape_sweep.py > gpurun_out/desc_sweep.log 2>&1
