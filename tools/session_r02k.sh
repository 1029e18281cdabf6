# zero-copy staging A/B: host-path tests with CIR_ZERO_COPY=1, config 5 and config2host both ways
mkdir -p gpurun_out
CIR_ZERO_COPY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "host or file or scan or memory or sync or verify or check or split or golden or hash_bytes" > gpurun_out/pytest_zc.log 2>&1 || exit $?
for zc in 0 1; do
  CIR_ZERO_COPY=$zc CIR_TRACE=1 timeout -k 10 600 python bench.py --workload config5 --steps 3 --tree-gib 16 > gpurun_out/cfg5_zc$zc.json 2> gpurun_out/cfg5_zc$zc.err || exit $?
done
rm -rf /dev/shm/ciruela_bench_tree
for zc in 0 1; do
  CIR_ZERO_COPY=$zc timeout -k 10 400 python bench.py --workload config2host --steps 3 --host-gib 16 > gpurun_out/c2h_zc$zc.json 2> gpurun_out/c2h_zc$zc.err || exit $?
done
