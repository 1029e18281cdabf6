# chunk split correctness + shapes + config-3 traces at 1 / 4 contexts
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chunks" > gpurun_out/pytest_chunks.log 2>&1 || exit $?
for sh in 32768_16384 32768_32768 32768_32769 32768_49152 32768_49153 32768_65535 32768_65536 262144_32768 262144_49153 262144_65535 262144_65536 1048576_32768 4096_8388608; do
  set -- ${sh/_/ }
  timeout -k 10 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/shape.json 2> gpurun_out/shape.err || exit $?
  echo "bs=$1 nblk=$2 $(grep -o '"value": [0-9.]*' gpurun_out/shape.json) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/shape.json) $(grep -o '"parity": "[a-z]*"' gpurun_out/shape.json)" >> gpurun_out/shapes.log
done
for k in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qtrace$k -o run -- python3 tools/queue_probe.py --contexts $k --steps 3 > gpurun_out/qtrace$k.log 2>&1 || exit $?
done
