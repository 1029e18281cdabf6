#!/bin/bash
# Config 5 (one 50 GiB tree, kept between runs) at several reader counts
# (CIR_SCAN_THREADS; 0 = the library's choice), one process each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${THREADS:-4 8 0}; do
  CIR_SCAN_THREADS=$t timeout -k 10 400 python bench.py --workload config5 --steps 2 \
    --tree-gib "${TREE_GIB:-50}" --no-cpu-baseline > "gpurun_out/c5t_$t.json" \
    2> "gpurun_out/c5t_$t.err" || { rm -rf /dev/shm/ciruela_bench_tree; exit 1; }
  echo "== readers $t"
  python3 tools/cfg5_report.py "gpurun_out/c5t_$t.json" | head -3
done
rm -rf /dev/shm/ciruela_bench_tree
