# quad vs lane crossover after the hand-scheduled quad loop: chunk-form shapes
# with CIR_QUAD_SMALL_BATCH = 49153 (lane from 49153 blocks) and 2^30 (quad)
mkdir -p gpurun_out
rm -f gpurun_out/crossover.log
for sh in 32768_40960 32768_49152 32768_57344 32768_65535 32768_65536 32768_81920 32768_98304 32768_131072 262144_49152 262144_65536 262144_98304; do
  set -- ${sh/_/ }
  for t in 49153 1073741824; do
    CIR_QUAD_SMALL_BATCH=$t timeout -k 10 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/shape.json 2> gpurun_out/shape.err || exit $?
    echo "bs=$1 nblk=$2 thr=$t $(grep -o '"value": [0-9.]*' gpurun_out/shape.json) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/shape.json) $(grep -o '"parity": "[a-z]*"' gpurun_out/shape.json)" | tee -a gpurun_out/crossover.log
  done
done
