mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_quad.py abtest/base.so abtest/new.so > gpurun_out/abquad.log 2>&1 || exit $?
timeout -k 10 200 python tools/quad_probe.py > gpurun_out/quad_probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit $?
for k in 1 4; do
  timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/queue_probe.log 2>&1 || exit $?
  CIR_SHARED_PART_QUEUES=1 timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/queue_probe.log 2>&1 || exit $?
done
