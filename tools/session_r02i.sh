# 16-bit keys (onesweep): tests + config 3 at 1 / 4 contexts + a trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "desc or quad or verify or config3 or scan or host or golden" > gpurun_out/pytest_q.log 2>&1 || exit $?
for k in 1 4 1 4; do
  timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/keys16.log 2>&1 || exit $?
done
rm -rf gpurun_out/ktrace4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace4 -o run -- python3 tools/queue_probe.py --contexts 4 --steps 3 > gpurun_out/ktrace4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit $?
