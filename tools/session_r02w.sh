# bounded-grid key kernel: parity, config-3 trace, 1 / 4 contexts
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "desc or config3 or blocks or scan or host or verify or hash_bytes or golden" > gpurun_out/pytest_keys2.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_keys2.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3tr2 -o run -- python3 bench.py --workload config3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c3tr2.log 2>&1 || exit $?
rm -f gpurun_out/qp3.log
for r in 1 2; do for k in 1 4; do timeout -k 10 200 python tools/queue_probe.py --contexts $k --steps 10 2>&1 | grep -v amdgpu >> gpurun_out/qp3.log || exit $?; done; done
cat gpurun_out/qp3.log
