# hand-scheduled quad loop (quad_fast): parity, then A/B one library per process
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_fast.log 2>&1 || exit $?
tail -2 gpurun_out/pytest_fast.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config3 or quad" > gpurun_out/pytest_fast_full.log 2>&1 || exit $?
tail -2 gpurun_out/pytest_fast_full.log
bash tools/ab_proc.sh 3 abtest/fast0.so abtest/fast1.so > gpurun_out/ab_fast.log 2>&1
