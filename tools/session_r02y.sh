# lane pace after the ordering fixes: one process per pace
mkdir -p gpurun_out/pace4
for r in 1 2; do
  for p in 0 48 64 80 100; do
    CIR_LANE_PACE=$p timeout -k 10 300 python bench.py --workload config3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pace4/p${p}_r$r.json 2> gpurun_out/pace4/p${p}_r$r.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/pace4/p${p}_r$r.json').read().strip().splitlines()[-1]);print('pace $p', d['value'], d['ms_per_step'], d.get('matches_oracle'))"
  done
done
