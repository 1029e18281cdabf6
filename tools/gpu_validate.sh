set -o pipefail
mkdir -p gpurun_out/r6s2
cd /root/repo
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6s2/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6s2/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6s2/bench.json 2> gpurun_out/r6s2/bench.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r6s2/prof -o run -- python3 /root/repo/bench.py --gpus 1 --steps 20 --warmup 5 > /root/repo/gpurun_out/r6s2/bench_under_rocprof.json 2> /root/repo/gpurun_out/r6s2/bench_under_rocprof.err
