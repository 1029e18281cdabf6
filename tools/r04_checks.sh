#!/bin/bash
# Round-4 checks on one GPU box: the async verify and hash_bytes tests (with
# their printed timings), the C-thread hash_bytes probe, config 5 with both
# footers on an 8 GiB tree and config 5 split over three device states of
# the one GPU (CIR_DEBUG_SPLIT=3).  Each GPU step under its own timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s \
  -k "verify or hash_bytes" -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/async.log 2>&1 || { tail -20 gpurun_out/async.log; exit 1; }
tail -3 gpurun_out/async.log
grep -E "async verify|hash_bytes 32" gpurun_out/async.log
bash tools/gpu_session.sh hbconc || exit 1
timeout -k 10 400 python bench.py --workload config5 --steps 2 --tree-gib 8 --footer ab \
  --cpu-seconds 0.5 > gpurun_out/c5small.json 2> gpurun_out/c5small.err || exit 1
CIR_DEBUG_SPLIT=3 timeout -k 10 400 python bench.py --workload config5 --steps 2 --tree-gib 16 \
  --cpu-seconds 0.5 > gpurun_out/c5split.json 2> gpurun_out/c5split.err
rc=$?
rm -rf /dev/shm/ciruela_bench_tree
python3 tools/cfg5_report.py gpurun_out/c5small.json
python3 tools/cfg5_report.py gpurun_out/c5split.json
exit $rc
