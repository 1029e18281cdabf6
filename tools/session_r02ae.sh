# write-combined staging A/B: config 5 and config 2 from host memory
mkdir -p gpurun_out
for wc in 0 1 0 1; do
  CIR_STAGING_WC=$wc timeout -k 10 600 python bench.py --workload config5 --steps 3 --tree-gib 16 --no-cpu-baseline > gpurun_out/cfg5_wc$wc.json 2> gpurun_out/cfg5_wc$wc.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/cfg5_wc$wc.json').read().strip().splitlines()[-1]);print('cfg5 wc=$wc', d['value'], d.get('seconds_all'), d.get('matches_oracle'))"
  CIR_STAGING_WC=$wc timeout -k 10 400 python bench.py --workload config2host --steps 3 --host-gib 16 --no-cpu-baseline > gpurun_out/c2h_wc$wc.json 2> gpurun_out/c2h_wc$wc.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/c2h_wc$wc.json').read().strip().splitlines()[-1]);print('c2h wc=$wc', d['value'], d.get('matches_oracle'))"
done
rm -rf /dev/shm/ciruela_bench_tree
