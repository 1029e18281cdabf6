# HEAD validation: GPU suite, smoke, headline bench, config 3, config 2 SHA
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_head.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_head.log 2>&1
step bench 400 python bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
step cfg3 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3_head.json 2> gpurun_out/cfg3_head.err
step sha 300 python bench.py --workload config2sha --steps 5 > gpurun_out/sha_head.json 2> gpurun_out/sha_head.err
