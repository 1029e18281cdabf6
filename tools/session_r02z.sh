# SHA-512 asm rounds: parity (every sha test), then config-2 SHA bench: asm (default build) vs compiled
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sha or hidden or fixture or ht or rewrite" > gpurun_out/pytest_sha.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_sha.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload config2sha --steps 5 --no-cpu-baseline > gpurun_out/sha_asm_r$r.json 2> gpurun_out/sha_asm_r$r.err || exit $?
  CIRUELA_AMD_LIB=$PWD/abtest/sha0.so timeout -k 10 300 python bench.py --workload config2sha --steps 5 --no-cpu-baseline > gpurun_out/sha_c_r$r.json 2> gpurun_out/sha_c_r$r.err || exit $?
  for v in asm c; do python3 -c "import json;d=json.loads(open('gpurun_out/sha_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v', d['value'], d.get('ms_per_step'), d.get('matches_oracle'))"; done
done
