# config 3: quad / lane kernel durations vs lane-part grid cap (rocprofv3 kernel trace)
mkdir -p gpurun_out/lanecap
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cap in 96 128 160 192 224 320 0; do
  CIR_LANE_WG=$cap timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lanecap/c$cap -o run -- python bench.py --workload config3 --steps 6 --warmup 2 > gpurun_out/lanecap/c$cap.log 2>&1 || exit $?
done
