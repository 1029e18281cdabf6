# Relays from concurrent callers, plus the relay / descriptor tests.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "concurrent or relay" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conc.log 2>&1
