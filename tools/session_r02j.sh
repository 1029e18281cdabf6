# early quad start: tests + A/B + contexts probe
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "desc or quad or verify or config3 or scan or host or golden or hash_bytes or memory" > gpurun_out/pytest_q.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_quad.py abtest/late_base.so abtest/early.so > gpurun_out/abquad_early.log 2>&1 || exit $?
for k in 1 4 1 4; do
  timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/early.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit $?
