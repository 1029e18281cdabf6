# A fresh process's HIP start-up under environment variants
# (build/hip_init_probe: each step's ms; the wall time includes the library
# load and exit), plus one AMD_LOG_LEVEL=4 run whose timestamps show where
# each stream's time goes, and the one-shot CLI on the config-1 tree.
# Usage (on the GPU box): bash tools/cli_start_env.sh [rounds=3]
set -e
rounds=${1:-3}
mkdir -p gpurun_out
echo "visible: HIP=${HIP_VISIBLE_DEVICES:-} ROCR=${ROCR_VISIBLE_DEVICES:-};" \
  "kfd nodes $(ls /sys/class/kfd/kfd/topology/nodes | wc -l); render nodes $(ls /dev/dri | tr '\n' ' ')"
run() {  # label, env...
  local label=$1; shift
  s=$(date +%s%N)
  out=$(env "$@" timeout -k 5 60 ./build/hip_init_probe 2>&1) || true
  e=$(date +%s%N)
  echo "$label $(( (e - s) / 1000000 )) ms | $out"
}
# back to back, then with a 1 s gap (does the previous process's exit slow
# the next one's start?)
for i in $(seq 1 4); do run back2back X=1; done
for i in $(seq 1 4); do sleep 1; run gap1s X=1; done
for i in $(seq 1 "$rounds"); do
  for v in HSA_ENABLE_INTERRUPT=0 HSA_DISABLE_IMAGE=1 HSA_DISCOVER_COPY_AGENTS=0 \
           HSA_DISABLE_PC_SAMPLING=1 ROC_AQL_QUEUE_SIZE=1024 HSA_KERNARG_POOL_SIZE=262144 \
           HIP_ENABLE_DEFERRED_LOADING=0 GPU_STAGING_BUFFER_SIZE=1 HSA_TOOLS_DISABLE_REGISTER=1; do
    sleep 1
    run "$v" "$v"
  done
done
AMD_LOG_LEVEL=4 timeout -k 5 60 ./build/hip_init_probe > gpurun_out/amdlog_probe.txt 2>&1 || true
echo "amd log: $(wc -l < gpurun_out/amdlog_probe.txt) lines"
python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.make_config1_tree('/tmp/c1tree')"
cli() {
  s=$(date +%s%N)
  CIR_TRACE=1 timeout -k 5 60 ./bin/ciruela-index sync --append /tmp/c1tree:/b > /dev/null \
    2> gpurun_out/cli_env.err
  e=$(date +%s%N)
  echo "cli $1 $(( (e - s) / 1000000 )) ms | $(grep -E 'HIP runtime start|cir_init [0-9]' gpurun_out/cli_env.err | tr '\n' ' ')"
}
for i in $(seq 1 6); do cli back2back; done
for i in $(seq 1 4); do sleep 1; cli gap1s; done
