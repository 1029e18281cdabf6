mkdir -p gpurun_out/r6sweep
CIR_SCAN_SWEEP_SEEDS=400 CIR_SCAN_SWEEP_FIRST=120000 CIR_HOST_SWEEP_SEEDS=300 CIR_HOST_SWEEP_FIRST=130000 CIR_SWEEP_SEEDS=200 CIR_SWEEP_FIRST=140000 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 800 --timeout-method thread -k 'randomized_scan_sweep or randomized_host_sweep or test_randomized_sweep' > gpurun_out/r6sweep/sweep.log 2>&1
