#!/bin/bash
# The scan's round-robin stripes over several devices, on one GPU box: the
# split and randomized scan tests (plus SWEEP more random seeds), then
# config 5 split over three device states of the one GPU (CIR_DEBUG_SPLIT=3,
# 16 GiB tree) and unsplit (8 GiB).  Each GPU step under its own timeout.
#   bash tools/stripe_check.sh [SWEEP=40]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP=${1:-40}
CIR_SCAN_SWEEP_SEEDS=$SWEEP timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu \
  -x -q -s -k "split_paths or randomized_scan" -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/stripe_tests.log 2>&1 \
  || { tail -30 gpurun_out/stripe_tests.log; exit 1; }
tail -2 gpurun_out/stripe_tests.log
CIR_DEBUG_SPLIT=3 timeout -k 10 400 python bench.py --workload config5 --steps 2 --tree-gib 16 \
  --cpu-seconds 0.5 > gpurun_out/c5split.json 2> gpurun_out/c5split.err || exit 1
timeout -k 10 400 python bench.py --workload config5 --steps 2 --tree-gib 8 \
  --cpu-seconds 0.5 > gpurun_out/c5one.json 2> gpurun_out/c5one.err
rc=$?
rm -rf /dev/shm/ciruela_bench_tree
python3 tools/cfg5_report.py gpurun_out/c5split.json
python3 tools/cfg5_report.py gpurun_out/c5one.json
exit $rc
