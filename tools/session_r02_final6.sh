# Validation of the final build: GPU suite, smoke, bench, config 3, and the
# descriptor / chunk shapes around the relay caps.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu6.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke6.log 2>&1
step bench 400 python bench.py > gpurun_out/bench6.json 2> gpurun_out/bench.err
step cfg3 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3_6.json 2> gpurun_out/cfg3.err
SWEEP_DESC=1 SWEEP_ONLY="4096:73728,4096:106496,2048:139264,4096:16384,32768:16384,32768:20480,32768:24576,32768:32768,32768:40960,1048576:20000,32768:65536,32768:65537,32768:98304,32768:98305,32768:131072,32768:131073" step desc 300 python -u tools/shape_sweep.py > gpurun_out/final6_desc.log 2>&1
step sweep 400 python -u tools/shape_sweep.py > gpurun_out/final6_chunks.log 2>&1
