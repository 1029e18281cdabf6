# static lane kernel back for unpaced batches: parity, lane-only, quad probe, config 3
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "desc or config3 or blocks or scan or host or verify or sha" > gpurun_out/pytest_split.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_split.log
timeout -k 10 120 python tools/lane_only_probe.py 2>&1 | grep lane-only | tail -3
timeout -k 10 200 python tools/quad_probe.py 2>&1 | grep -v amdgpu
for r in 1 2; do timeout -k 10 300 python bench.py --workload config3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3s.json 2>/dev/null || exit $?; python3 -c "import json;d=json.loads(open('gpurun_out/c3s.json').read().strip().splitlines()[-1]);print('config3', d['value'], d['ms_per_step'], d.get('matches_oracle'))"; done
