#!/bin/bash
# config 5 (e2e scan) pinned to each NUMA node of the box vs unpinned.
# Usage (on the GPU box): bash tools/numa_cfg5.sh [TREE_GIB]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
G=${1:-16}
run() {  # label cmd...
  local label=$1; shift
  timeout -k 10 600 "$@" python bench.py --workload config5 --steps 3 --tree-gib "$G" \
    > gpurun_out/numa_$label.json 2> gpurun_out/numa_$label.err
  local rc=$?
  echo "$label rc=$rc $(grep -o '"value": [0-9.]*\|"seconds_all": \[[0-9., ]*\]' gpurun_out/numa_$label.json | tr '\n' ' ')"
  rm -rf /dev/shm/ciruela_bench_tree
  [ $rc -eq 0 ] || exit $rc
}
N0=$(cat /sys/devices/system/node/node0/cpulist)
N1=$(cat /sys/devices/system/node/node1/cpulist)
run none
run node0 taskset -c "$N0"
run node1 taskset -c "$N1"
