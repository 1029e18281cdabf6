# self-contained fast quad block: parity, then layout-robustness A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_fast2.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_fast2.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config3 or quad" > gpurun_out/pytest_fast2_full.log 2>&1 || exit $?
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_fast2_full.log | tail -4
bash tools/ab_proc.sh 2 abtest/b0p0.so abtest/b1p0.so abtest/b0p3.so abtest/b1p3.so abtest/b1p6.so abtest/b1p9.so > gpurun_out/ab_fast2.log 2>&1
