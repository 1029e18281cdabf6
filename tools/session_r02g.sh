# k_gate instead of the timed k_delay: tests + config 3 at 1 / 4 contexts
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "desc or quad or verify or config3 or scan" > gpurun_out/pytest_q.log 2>&1 || exit $?
for k in 1 4 1 4; do
  timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/gate.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit $?
