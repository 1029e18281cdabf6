# quad-part lead time at 1 / 4 contexts (config 3)
mkdir -p gpurun_out
for r in 6 30 90; do
  for k in 1 4; do
    CIR_QUAD_LEAD_ROUNDS=$r timeout -k 10 200 python tools/queue_probe.py --contexts $k >> gpurun_out/lead.log 2>&1 || exit $?
    echo "lead_rounds=$r" >> gpurun_out/lead.log
  done
done
