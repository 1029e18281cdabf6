# One-shot `ciruela-index sync` of the config-1 tree (100 files, 10 MiB) in
# alternating processes: the CLI's default (blit copies below one staging
# slot) against SDMA copies forced with HSA_ENABLE_SDMA=1; CIR_TRACE gives the
# start-up steps.  Usage (on the GPU box): bash tools/cli_sdma_ab.sh [rounds=6]
set -e
rounds=${1:-6}
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.make_config1_tree('/tmp/c1tree')"
for i in $(seq 1 "$rounds"); do
  for mode in default sdma; do
    if [ $mode = sdma ]; then export HSA_ENABLE_SDMA=1; else unset HSA_ENABLE_SDMA; fi
    s=$(date +%s.%N)
    CIR_TRACE=1 timeout -k 5 60 ./bin/ciruela-index sync --append /tmp/c1tree:/b > /dev/null \
      2> "gpurun_out/cli_${mode}_$i.err"
    e=$(date +%s.%N)
    echo "$mode $(python3 -c "print(round(($e-$s)*1000,1))") ms | $(grep -E 'copies|HIP runtime start|first uploads|cir_init [0-9]' "gpurun_out/cli_${mode}_$i.err" | tr '\n' ' ')"
  done
done
