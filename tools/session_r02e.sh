# partial-wave uniform body: chunk tests, shapes, config-2 bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chunks or config2 or config4" > gpurun_out/pytest_chunks.log 2>&1 || exit $?
for sh in 32768_65535 32768_65536 32768_65472 32768_65473 262144_65535 262144_65536 262144_65472 4096_8388607; do
  set -- ${sh/_/ }
  timeout -k 10 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/shape.json 2> gpurun_out/shape.err || exit $?
  echo "bs=$1 nblk=$2 $(grep -o '"value": [0-9.]*' gpurun_out/shape.json) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/shape.json) $(grep -o '"parity": "[a-z]*"' gpurun_out/shape.json)" >> gpurun_out/shapes.log
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
