# kernel traces of config 3 at 1 and 4 contexts per process (hiq part streams)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qtrace$k -o run -- python3 tools/queue_probe.py --contexts $k --steps 3 > gpurun_out/qtrace$k.log 2>&1 || exit $?
done
