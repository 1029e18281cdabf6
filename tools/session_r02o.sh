# quad compression with the next line's LDS reads inside the asm block:
# parity (default build = RDI on), then one library per process A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_rdi.log 2>&1 || exit $?
tail -2 gpurun_out/pytest_rdi.log
bash tools/ab_proc.sh 3 abtest/rdi0.so abtest/rdi1.so > gpurun_out/ab_rdi.log 2>&1
