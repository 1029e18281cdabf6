#!/bin/bash
# cir_scan_v1_write (the index written out as it goes) against cir_scan_v1
# (whole buffer, copied out after the scan), on one GPU box: the scan
# parity tests that cover both (plus SWEEP random seeds), then config 5 on
# a TREE_GIB tree in alternating processes, ROUNDS pairs.  Each GPU step
# under its own timeout.
#   bash tools/scan_output_ab.sh [SWEEP=40] [TREE_GIB=50] [ROUNDS=2]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/scan_output_ab
SWEEP=${1:-40}
GIB=${2:-50}
ROUNDS=${3:-2}
CIR_SCAN_SWEEP_SEEDS=$SWEEP timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu \
  -x -q -s -k "written_as_it_goes or writer_failure or randomized_scan or long_index or split_paths" \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/scan_output_ab/tests.log 2>&1 \
  || { tail -30 gpurun_out/scan_output_ab/tests.log; exit 1; }
tail -2 gpurun_out/scan_output_ab/tests.log
rc=0
for r in $(seq 1 "$ROUNDS"); do
  for m in write buffer; do
    timeout -k 10 400 python bench.py --workload config5 --steps 3 --tree-gib "$GIB" \
      --no-cpu-baseline --scan-output $m > gpurun_out/scan_output_ab/c5_${m}_$r.json \
      2> gpurun_out/scan_output_ab/c5_${m}_$r.err || { rc=$?; break 2; }
    python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=r['phases_best']
print('%-6s round %s: %.2f GiB/s best (%s), first %.2f, matches_oracle %s, loop %.0f ms, tail %.2f ms' % (
  r.get('scan_output'), sys.argv[2], r['value'], r['seconds_all'], r['value_first'], r['matches_oracle'],
  b['phases_ms']['hash_loop_ms'], b['phases_ms']['footer_tail_ms']))" gpurun_out/scan_output_ab/c5_${m}_$r.json $r
  done
done
rm -rf /dev/shm/ciruela_bench_tree
exit $rc
