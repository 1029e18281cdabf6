# key-kernel wave reductions + idle-helper exit: parity, trace, config 3 at 1 / 4 contexts
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "desc or config3 or blocks or scan or host" > gpurun_out/pytest_keys.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_keys.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qtr1b -o run -- python3 tools/queue_probe.py --contexts 1 --steps 5 > gpurun_out/qtr1b.log 2>&1 || exit $?
rm -f gpurun_out/qp2.log
for r in 1 2; do for k in 1 4; do timeout -k 10 200 python tools/queue_probe.py --contexts $k --steps 10 2>&1 | grep -v amdgpu >> gpurun_out/qp2.log || exit $?; done; done
cat gpurun_out/qp2.log
