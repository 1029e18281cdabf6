# counting-sort ordering: parity, then config 3 at 1 / 4 contexts, counting sort vs hipCUB
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "not config2_full and not config4" > gpurun_out/pytest_csort.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_csort.log
rm -f gpurun_out/qp5.log
for r in 1 2; do for v in cub0 cub1; do for k in 1 4; do echo -n "$v " >> gpurun_out/qp5.log; CIRUELA_AMD_LIB=$PWD/abtest/$v.so timeout -k 10 200 python tools/queue_probe.py --contexts $k --steps 10 2>&1 | grep -v amdgpu >> gpurun_out/qp5.log || exit $?; done; done; done
cat gpurun_out/qp5.log
