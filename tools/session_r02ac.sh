# lane-only batches: counting-sort order vs hipCUB's stable order (pace 0: no helper)
mkdir -p gpurun_out
rm -f gpurun_out/lane_only_ab.log
for r in 1 2; do for v in cub0 cub1; do
  echo "== $v shuffled (config-3 offsets)" >> gpurun_out/lane_only_ab.log
  CIR_LANE_PACE=0 CIRUELA_AMD_LIB=$PWD/abtest/$v.so timeout -k 10 120 python tools/lane_only_probe.py 2>&1 | grep lane-only | tail -3 >> gpurun_out/lane_only_ab.log || exit $?
  echo "== $v unshuffled (quad_probe)" >> gpurun_out/lane_only_ab.log
  CIR_LANE_PACE=0 CIRUELA_AMD_LIB=$PWD/abtest/$v.so timeout -k 10 200 python tools/quad_probe.py 2>&1 | grep "lane only" >> gpurun_out/lane_only_ab.log || exit $?
done; done
cat gpurun_out/lane_only_ab.log
