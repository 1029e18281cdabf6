# Round-2 refresh after the relay: GPU suite, smoke, bench, full shape sweep
# with and without the relay.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step bench 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
CIR_RELAY=0 step sweep_off 400 python -u tools/shape_sweep.py > gpurun_out/sweep_off.log 2>&1
step sweep_on 400 python -u tools/shape_sweep.py > gpurun_out/sweep_on.log 2>&1
