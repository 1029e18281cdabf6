# lane pacing with dynamic tiles + helper: parity, then one process per pace
mkdir -p gpurun_out/pace2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "desc or config3" > gpurun_out/pytest_pace.log 2>&1 || exit $?
tail -2 gpurun_out/pytest_pace.log
for r in 1 2; do
  for p in 0 40 44 48 52 60 80; do
    CIR_LANE_PACE=$p timeout -k 10 300 python bench.py --workload config3 --steps 10 --warmup 3 > gpurun_out/pace2/p${p}_r$r.json 2> gpurun_out/pace2/p${p}_r$r.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/pace2/p${p}_r$r.json').read().strip().splitlines()[-1]);print('pace $p', d['value'], d['ms_per_step'])"
  done
done
