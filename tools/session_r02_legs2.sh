# Round-2 measurement session B (refresh): headline bench (with PMC traffic
# from profiles/pmc_traffic.json), secondary legs, the N>1 path rehearsed with
# two gloo ranks sharing the one GPU, hash_bytes latency, config 5.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$t" "$@"; local rc=$?
  echo "== $name rc=$rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step bench 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
step cfg1 200 python bench.py --workload config1 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err
step cfg3 300 python bench.py --workload config3 --steps 10 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err
step cfg2host 400 python bench.py --workload config2host --steps 3 > gpurun_out/cfg2host.json 2> gpurun_out/cfg2host.err
step cfg2sha 300 python bench.py --workload config2sha --steps 5 > gpurun_out/cfg2sha.json 2> gpurun_out/cfg2sha.err
step dist2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --blocks 262144 --steps 5 --warmup 1 > gpurun_out/dist2.json 2> gpurun_out/dist2.err
step latency 120 python tools/hash_bytes_latency.py > gpurun_out/latency.log 2>&1
step cfg5 900 python bench.py --workload config5 --steps 3 > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
rm -rf /dev/shm/ciruela_bench_tree
