# queue placement A/B: config 3 at 1 and 4 contexts per process, three part-stream modes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "desc or quad or verify" > gpurun_out/pytest_q.log 2>&1 || exit $?
for mode in hiq own2 plain; do
  for k in 1 4; do
    CIR_PART_STREAMS=$mode timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/queue_probe.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit $?
