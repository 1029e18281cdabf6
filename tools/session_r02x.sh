# early quad start: parity, config 3 at 1 / 4 contexts with and without it
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "desc or config3 or blocks or scan or host or verify or hash_bytes or golden" > gpurun_out/pytest_early.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_early.log
rm -f gpurun_out/qp4.log
for r in 1 2; do for eq in 1 0; do for k in 1 4; do echo -n "early=$eq " >> gpurun_out/qp4.log; CIR_EARLY_QUAD=$eq timeout -k 10 200 python tools/queue_probe.py --contexts $k --steps 10 2>&1 | grep -v amdgpu >> gpurun_out/qp4.log || exit $?; done; done; done
cat gpurun_out/qp4.log
