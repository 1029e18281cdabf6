#!/bin/bash
# Persistent host worker pool (HEAD) against per-batch threads (a build of
# the previous commit at abtest/libciruela_nopool.so, loaded through
# CIRUELA_AMD_LIB) in alternating processes: the scan and host-path parity
# tests on HEAD (plus SWEEP seeds), then config 5 (50 GiB and 1 GiB trees)
# and config 2 from host memory, ROUNDS pairs.  Each GPU step under its own
# timeout.
#   bash tools/pool_ab.sh [SWEEP=40] [ROUNDS=2]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/pool_ab
mkdir -p $out
SWEEP=${1:-40}
ROUNDS=${2:-2}
OLD=abtest/libciruela_nopool.so
CIR_SCAN_SWEEP_SEEDS=$SWEEP CIR_HOST_SWEEP_SEEDS=$SWEEP timeout -k 10 500 python -u -m pytest \
  tests/test_gpu_parity.py -m gpu -x -q -s -p no:cacheprovider --timeout 400 \
  --timeout-method thread -k "randomized or split_paths or hash_file or hash_memory or pipe or long_index or written or verify or hash_blocks" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
summ() {
  python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-14s %-6s round %s: %.3f GiB/s best %s matches_oracle %s' % (sys.argv[2], sys.argv[3],
  sys.argv[4], r['value'], r.get('seconds_all'), r.get('matches_oracle')))" "$@"
}
run() {  # lib label workload args...
  local lib=$1 label=$2 name=$3; shift 3
  if [ "$lib" = new ]; then
    timeout -k 10 400 python bench.py "$@" --no-cpu-baseline > $out/${name}_${label}.json 2> $out/${name}_${label}.err
  else
    CIRUELA_AMD_LIB=$OLD timeout -k 10 400 python bench.py "$@" --no-cpu-baseline > $out/${name}_${label}.json 2> $out/${name}_${label}.err
  fi
}
for r in $(seq 1 "$ROUNDS"); do
  for lib in new old; do
    run $lib ${lib}_$r c5 --workload config5 --steps 3 --tree-gib 50 || exit 1
    summ $out/c5_${lib}_$r.json config5-50G $lib $r
    run $lib ${lib}_$r c2h --workload config2host --steps 3 || exit 1
    summ $out/c2h_${lib}_$r.json config2host $lib $r
  done
done
rm -rf /dev/shm/ciruela_bench_tree
for r in $(seq 1 "$ROUNDS"); do
  for lib in new old; do
    run $lib ${lib}_$r c5s --workload config5 --steps 8 --tree-gib 1 || exit 1
    summ $out/c5s_${lib}_$r.json config5-1G $lib $r
  done
done
rm -rf /dev/shm/ciruela_bench_tree
