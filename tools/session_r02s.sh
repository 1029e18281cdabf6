# fast loop in k_chain_step / k_single: parity + hash_bytes latency
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_single.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_single.log
timeout -k 10 300 python tools/hash_bytes_latency.py > gpurun_out/latency_fast.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/latency_fast.log
