# Round-2 measurement session A: GPU suite, headline bench, rocprof kernel
# stats and PMC passes (one counter group per pass).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$t" "$@"; local rc=$?
  echo "== $name rc=$rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step bench 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES; do
  step "pmc_$c" 120 rocprofv3 --pmc "$c" --output-format csv -d "gpurun_out/pmc_$c" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "gpurun_out/pmc_$c.log" 2>&1
done
