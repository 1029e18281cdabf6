mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 4; do
  rm -rf gpurun_out/gtrace$k
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gtrace$k -o run -- python3 tools/queue_probe.py --contexts $k --steps 3 > gpurun_out/gtrace$k.log 2>&1 || exit $?
done
