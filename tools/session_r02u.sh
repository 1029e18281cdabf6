# quad band for fractional lane waves: parity + the crossover shapes with the default rule
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunks" > gpurun_out/pytest_band.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_band.log
rm -f gpurun_out/crossover_rule.log
for sh in 32768_49152 32768_49153 32768_65535 32768_65536 32768_65537 32768_81920 32768_98304 32768_106496 32768_106497 32768_131072 262144_65536 262144_98304; do
  set -- ${sh/_/ }
  timeout -k 10 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/shape.json 2> gpurun_out/shape.err || exit $?
  echo "bs=$1 nblk=$2 $(grep -o '"value": [0-9.]*' gpurun_out/shape.json) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/shape.json) $(grep -o '"parity": "[a-z]*"' gpurun_out/shape.json)" | tee -a gpurun_out/crossover_rule.log
done
