#!/bin/bash
# The staged paths' batch ramp (first batches 1/8, 1/4, 1/2 of a slot) on
# and off (CIR_STAGE_RAMP=0) in alternating processes: the scan and host-path
# parity tests (plus SWEEP random seeds each) with the ramp, then config 5
# (TREE_GIB tree) and config 2 from host memory, ROUNDS pairs each.  Each GPU
# step under its own timeout.
#   bash tools/ramp_ab.sh [SWEEP=40] [TREE_GIB=50] [ROUNDS=2]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ramp_ab
mkdir -p $out
SWEEP=${1:-40}
GIB=${2:-50}
ROUNDS=${3:-2}
CIR_SCAN_SWEEP_SEEDS=$SWEEP CIR_HOST_SWEEP_SEEDS=$SWEEP timeout -k 10 500 python -u -m pytest \
  tests/test_gpu_parity.py -m gpu -x -q -s -p no:cacheprovider --timeout 400 \
  --timeout-method thread -k "randomized or split_paths or hash_file or hash_memory or pipe or long_index or written" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
summ() {
  python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-10s ramp=%s round %s: %.3f GiB/s best %s first %s matches_oracle %s' % (sys.argv[3], sys.argv[2],
  sys.argv[4], r['value'], r.get('seconds_all'), r.get('value_first'), r.get('matches_oracle')))" "$@"
}
for r in $(seq 1 "$ROUNDS"); do
  for ramp in 1 0; do
    CIR_STAGE_RAMP=$ramp timeout -k 10 400 python bench.py --workload config5 --steps 3 \
      --tree-gib "$GIB" --no-cpu-baseline > $out/c5_${ramp}_$r.json 2> $out/c5_${ramp}_$r.err || exit 1
    summ $out/c5_${ramp}_$r.json $ramp config5 $r
    CIR_STAGE_RAMP=$ramp timeout -k 10 300 python bench.py --workload config2host --steps 3 \
      --no-cpu-baseline > $out/c2h_${ramp}_$r.json 2> $out/c2h_${ramp}_$r.err || exit 1
    summ $out/c2h_${ramp}_$r.json $ramp config2host $r
  done
done
rm -rf /dev/shm/ciruela_bench_tree
