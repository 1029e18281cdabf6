# config 3: lane-part grid cap sweep (does a narrower, longer lane part keep
# the quad part's clock up?).  One process per setting; then kernel stats
# for cap 0 and cap 224.
mkdir -p gpurun_out
for cap in 384 320 256 224 192 160 128 0; do
  CIR_LANE_WG=$cap timeout -k 10 300 python bench.py --workload config3 --steps 10 --warmup 3 > gpurun_out/cfg3_lanecap$cap.json 2> gpurun_out/cfg3_lanecap$cap.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/cfg3_lanecap$cap.json').read().strip().splitlines()[-1]);print('cap $cap', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cap in 0 224; do
  CIR_LANE_WG=$cap timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lanecap$cap -o run -- python bench.py --workload config3 --steps 10 --warmup 3 > gpurun_out/prof_lanecap$cap.log 2>&1 || exit $?
done
