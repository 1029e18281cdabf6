#!/bin/bash
# Experiment: lane/quad split for medium chunk batches (CIR_HYBRID_K blocks in
# quad mode, the rest in lane mode, concurrently).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sh in 32768_65536 32768_98304 32768_131072 262144_65536 262144_98304; do
  set -- ${sh/_/ }
  for k in 0 8192 16384 24576; do
    CIR_HYBRID_K=$k timeout -k 10 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 \
      --no-cpu-baseline > gpurun_out/hyb.json 2> gpurun_out/hyb.err || exit 1
    echo "bs=$1 nblk=$2 k=$k $(grep -o '"value": [0-9.]*' gpurun_out/hyb.json) $(grep -o '"parity": "[a-z]*"' gpurun_out/hyb.json)"
  done
done
