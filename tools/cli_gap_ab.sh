# Does a one-shot `ciruela-index sync` start slower right after another GPU
# process exits?  The config-1 tree synced N times back to back and N times
# with a pause before each run, alternating blocks of 5; CIR_TRACE gives each
# run's device discovery ("HIP runtime start") and cir_init.
# Usage (on the GPU box): bash tools/cli_gap_ab.sh [n=20] [pause=0.5]
set -e
n=${1:-20}
pause=${2:-0.5}
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.make_config1_tree('/tmp/c1tree')"
one() {
  s=$(date +%s%N)
  CIR_TRACE=1 timeout -k 5 60 ./bin/ciruela-index sync --append /tmp/c1tree:/b > /dev/null \
    2> gpurun_out/cli_gap.err
  e=$(date +%s%N)
  echo "$1 $(( (e - s) / 1000000 )) ms | $(grep -oE 'HIP runtime start [0-9.]+ ms|cir_init [0-9.]+ ms' gpurun_out/cli_gap.err | tr '\n' ' ')"
}
for b in $(seq 1 $(( n / 5 ))); do
  for i in 1 2 3 4 5; do one back2back; done
  for i in 1 2 3 4 5; do sleep "$pause"; one "pause$pause"; done
done
