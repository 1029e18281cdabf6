#!/bin/bash
# One GPU session on the gpurun box: each GPU step under its own timeout,
# stop at the first step that faults / aborts / times out (rc other than
# 0 or 1).  Usage: tools/gpu_session.sh STEP...   (steps: smoke tests bench
# prof pmc ubench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

step() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)" >&2
    exit $rc
  fi
  return 0
}

for s in "$@"; do
  case "$s" in
    ablib)
      step ablib 600 python tools/ab_lib.py abtest/*.so > gpurun_out/ablib.log 2>&1
      cat gpurun_out/ablib.log ;;
    abquad)
      step abquad 600 python tools/ab_quad.py abtest/*.so > gpurun_out/abquad.log 2>&1
      cat gpurun_out/abquad.log ;;
    abquadtrace)  # kernel trace of ab_quad.py over the first abtest/*.so only
      lib=$(ls abtest/*.so | head -1)
      step abquadtrace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abqt \
        -o run -- python3 tools/ab_quad.py "$lib" > gpurun_out/abquadtrace.log 2>&1
      cat gpurun_out/abquadtrace.log | grep -v amdgpu.ids ;;
    cfg5blit)
      HSA_ENABLE_SDMA=0 step cfg5blit 1000 python bench.py --workload config5 --steps 3 \
        --tree-gib "${TREE_GIB:-50}" > gpurun_out/cfg5blit.json 2> gpurun_out/cfg5blit.err
      rm -rf /dev/shm/ciruela_bench_tree
      cat gpurun_out/cfg5blit.json ;;
    cli)
      head -c 100000 /dev/urandom > /tmp/cli_probe.bin
      step cli 120 ./bin/ciruela-index hash /tmp/cli_probe.bin ;;
    smoke)
      step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    sanitizers)  # the host code under ASan + UBSan and under TSan (make builds both drivers)
      ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 step asan 400 \
        ./build/host_asan_driver "${SAN_ROUNDS:-60}" "${SAN_SEED:-1}" > gpurun_out/asan.out 2> gpurun_out/asan.err
      TSAN_OPTIONS="suppressions=tools/tsan_hip.supp report_thread_leaks=0" step tsan 600 \
        ./build/host_tsan_driver "${SAN_ROUNDS:-30}" "${SAN_SEED:-1}" > gpurun_out/tsan.out 2> gpurun_out/tsan.err
      cat gpurun_out/asan.out gpurun_out/tsan.out
      echo "tsan warnings: $(grep -c 'WARNING: ThreadSanitizer' gpurun_out/tsan.err)" ;;
    tests)
      step tests 1100 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider \
        --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
        --junitxml=gpurun_out/pytest_gpu.xml > gpurun_out/pytest_gpu.log 2>&1
      grep -E "PASS|FAIL|ERROR|SKIP" gpurun_out/pytest_gpu.log | tail -15
      tail -3 gpurun_out/pytest_gpu.log ;;
    dist2)  # bench.py launching two ranks itself (gloo: they share the one GPU)
      step dist2 600 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 \
        --blocks "${DIST_BLOCKS:-262144}" > gpurun_out/dist2.json 2> gpurun_out/dist2.err
      cat gpurun_out/dist2.json ;;
    dist4)  # bench.py launching four ranks itself (gloo: they share the one GPU)
      step dist4 600 python bench.py --gpus 4 --dist-backend gloo --steps 5 --warmup 1 \
        --blocks "${DIST_BLOCKS:-262144}" > gpurun_out/dist4.json 2> gpurun_out/dist4.err
      cat gpurun_out/dist4.json ;;
    bench)  # the driver's command
      step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json \
        2> gpurun_out/bench.err
      cat gpurun_out/bench.json ;;
    forcedist)  # the N>1 code path (process group over RCCL, config 4) on one self-launched rank
      step forcedist 600 python3 bench.py --gpus 1 --force-dist --steps 20 --warmup 3 \
        > gpurun_out/forcedist.json 2> gpurun_out/forcedist.err
      cat gpurun_out/forcedist.json ;;
    cfg5footer)  # config 5 with the footer on the host thread and on the GPU chain, alternating
      step cfg5footer 900 python bench.py --workload config5 --footer "${FOOTER:-ab}" \
        --steps "${STEPS:-3}" --tree-gib "${TREE_GIB:-50}" --hash "${HASH:-blake2b}" \
        > gpurun_out/cfg5footer.json 2> gpurun_out/cfg5footer.err
      rm -rf /dev/shm/ciruela_bench_tree
      python3 tools/cfg5_report.py gpurun_out/cfg5footer.json ;;
    cfg5copy)  # config 5 with the readers' two copy modes, alternating processes, one tree
      for rep in $(seq 1 "${REPS:-2}"); do
        for mode in direct nt; do
          CIR_STAGE_COPY=$mode step "cfg5copy_$mode" 600 python bench.py --workload config5 \
            --steps "${STEPS:-3}" --tree-gib "${TREE_GIB:-50}" --no-cpu-baseline \
            > "gpurun_out/cfg5copy_${mode}_$rep.json" 2> "gpurun_out/cfg5copy_${mode}_$rep.err"
          echo "== $mode rep $rep"
          python3 tools/cfg5_report.py "gpurun_out/cfg5copy_${mode}_$rep.json"
        done
      done
      rm -rf /dev/shm/ciruela_bench_tree ;;
    c2hcopy)  # config 2 from host memory with the two staging copy modes, alternating processes
      for rep in $(seq 1 "${REPS:-2}"); do
        for mode in direct nt; do
          CIR_STAGE_COPY=$mode step "c2h_$mode" 600 python bench.py --workload config2host --steps 3 \
            --host-gib "${HOST_GIB:-32}" --cpu-seconds 0.5 > "gpurun_out/c2hcopy_${mode}_$rep.json" \
            2> "gpurun_out/c2hcopy_${mode}_$rep.err"
          echo "c2h $mode rep $rep $(grep -o '"value": [0-9.]*\|"seconds_all": \[[0-9., ]*\]\|"matches_oracle": [a-z]*' "gpurun_out/c2hcopy_${mode}_$rep.json" | head -3 | tr '\n' ' ')"
        done
      done ;;
    cfg2sha)
      step cfg2sha 600 python bench.py --workload config2sha --steps 10 --warmup 2 \
        > gpurun_out/cfg2sha.json 2> gpurun_out/cfg2sha.err
      cat gpurun_out/cfg2sha.json ;;
    crossover)  # cir_verify_blocks batch vs the drop-in vs one host core, 32 KiB blocks
      step crossover 300 python tools/verify_crossover.py > gpurun_out/crossover.log 2>&1
      cat gpurun_out/crossover.log ;;
    hbconc)  # concurrent drop-in callers from C threads
      step hbconc 300 ./build/hash_bytes_conc 32768 64 > gpurun_out/hbconc.log 2>&1
      cat gpurun_out/hbconc.log ;;
    latency)
      step latency 300 python tools/hash_bytes_latency.py > gpurun_out/latency.log 2>&1
      cat gpurun_out/latency.log ;;
    sweep)  # the randomized parity cases over SWEEP_SEEDS more seeds
      CIR_SWEEP_SEEDS=${SWEEP_SEEDS:-40} CIR_SWEEP_FIRST=${SWEEP_FIRST:-7000} step sweep 900 \
        python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -k test_randomized_sweep \
        -p no:cacheprovider --timeout 850 --timeout-method thread > gpurun_out/sweep.log 2>&1
      tail -3 gpurun_out/sweep.log ;;
    bench_direct)
      step bench_direct 400 python bench.py --steps 10 --warmup 2 --loader direct \
        --no-cpu-baseline > gpurun_out/bench_direct.json 2> gpurun_out/bench_direct.err
      cat gpurun_out/bench_direct.json ;;
    prof)
      # the driver's own bench command, under the profiler
      step prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/prof.log 2>&1
      find gpurun_out/prof -name '*stats*' | head ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
               SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU; do
        step "pmc_$c" 600 rocprofv3 --pmc "$c" --output-format csv \
          -d "gpurun_out/pmc_$c" -o run -- python3 bench.py --steps 3 --warmup 1 \
          --no-cpu-baseline --no-secondary > "gpurun_out/pmc_$c.log" 2>&1
      done ;;
    pmct)  # HBM bytes of config 2's k_chunks (FETCH_SIZE and WRITE_SIZE, one pass each)
      for c in FETCH_SIZE WRITE_SIZE; do
        step "pmct_$c" 300 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/pmct_$c" -o run \
          -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
          > "gpurun_out/pmct_$c.log" 2>&1
      done ;;
    cfg3)
      step cfg3 600 python bench.py --workload config3 --steps 5 --warmup 1 \
        > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err
      cat gpurun_out/cfg3.json ;;
    prof3)
      step prof3 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof3 -o run -- python3 bench.py --workload config3 --steps 3 --warmup 1 \
        > gpurun_out/prof3.log 2>&1
      cat gpurun_out/prof3/run_kernel_stats.csv | cut -c1-200 ;;
    pmc3)  # SQ counters of config 3 per dispatch (k_quad_long's per-compression budget)
      i=0
      for c in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
               "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
               "SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"; do
        i=$((i+1))
        step "pmc3_$i" 300 rocprofv3 --pmc $c --output-format csv \
          -d "gpurun_out/pmc3_$i" -o run -- python3 bench.py --workload config3 --steps 2 \
          --warmup 1 > "gpurun_out/pmc3_$i.log" 2>&1
      done ;;
    pmc3t)  # HBM bytes of config 3's batches (FETCH_SIZE and WRITE_SIZE, one pass each)
      for c in FETCH_SIZE WRITE_SIZE; do
        step "pmc3t_$c" 300 rocprofv3 --pmc $c --output-format csv \
          -d "gpurun_out/pmc3t_$c" -o run -- python3 bench.py --workload config3 --steps 2 \
          --warmup 1 > "gpurun_out/pmc3t_$c.log" 2>&1
      done ;;
    pmcreq)  # read requests by size (the terms of FETCH_SIZE), config 2 and config 3
      step pmcreq_c2 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum \
        TCC_EA0_RDREQ_DRAM_sum --output-format csv -d gpurun_out/pmcreq_c2 -o run -- python3 bench.py \
        --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/pmcreq_c2.log 2>&1
      step pmcreq_c3 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum \
        TCC_EA0_RDREQ_DRAM_sum --output-format csv -d gpurun_out/pmcreq_c3 -o run -- python3 bench.py \
        --workload config3 --steps 2 --warmup 1 > gpurun_out/pmcreq_c3.log 2>&1 ;;
    firstread)
      step firstread 600 python tools/first_read_probe.py --gib "${TREE_GIB:-16}" \
        --read-first "${READ_FIRST:-1}" > gpurun_out/firstread.log 2>&1
      cat gpurun_out/firstread.log ;;
    cfg3ab)
      for lib in abtest/*.so; do
        CIRUELA_AMD_LIB=$PWD/$lib step "cfg3_$lib" 300 python bench.py --workload config3 --steps 5 --warmup 1 \
          > gpurun_out/cfg3ab.json 2> gpurun_out/cfg3ab.err
        echo "$lib $(cat gpurun_out/cfg3ab.json)"
      done ;;
    cfg5ab)  # config 5 (one tree, kept) and config 2 from host, alternating abtest/*.so
      for rep in $(seq 1 "${REPS:-2}"); do
        for lib in abtest/*.so; do
          CIRUELA_AMD_LIB=$PWD/$lib step "cfg5_$lib" 600 python bench.py --workload config5 --steps 3 \
            --tree-gib "${TREE_GIB:-32}" > gpurun_out/cfg5ab.json 2> gpurun_out/cfg5ab.err
          echo "cfg5 $rep $lib $(grep -o '"value": [0-9.]*\|"seconds_all": \[[0-9., ]*\]' gpurun_out/cfg5ab.json | head -2 | tr '\n' ' ')"
          [ -n "${CFG5_ONLY:-}" ] && continue
          CIRUELA_AMD_LIB=$PWD/$lib step "c2h_$lib" 600 python bench.py --workload config2host --steps 3 \
            --host-gib "${HOST_GIB:-16}" > gpurun_out/c2hab.json 2> gpurun_out/c2hab.err
          echo "c2h $rep $lib $(grep -o '"value": [0-9.]*\|"seconds_all": \[[0-9., ]*\]' gpurun_out/c2hab.json | head -2 | tr '\n' ' ')"
        done
      done
      rm -rf /dev/shm/ciruela_bench_tree ;;
    cfg2host)
      step cfg2host 600 python bench.py --workload config2host --steps 3 --host-gib "${HOST_GIB:-32}" \
        > gpurun_out/cfg2host.json 2> gpurun_out/cfg2host.err
      cat gpurun_out/cfg2host.json ;;
    shapes)
      for sh in ${SHAPES:-4096_8388608 131072_262144 1048576_32768 4194304_8192 32768_65535 32768_65536 32768_16384 262144_65535 262144_65536}; do
        set -- ${sh/_/ }
        step "bs$1" 300 python bench.py --block-size $1 --blocks $2 --steps 5 --warmup 1 --no-cpu-baseline \
          > gpurun_out/shape.json 2> gpurun_out/shape.err
        echo "bs=$1 nblk=$2 $(grep -o '"value": [0-9.]*' gpurun_out/shape.json) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/shape.json)"
      done ;;
    shapesab)  # SHAPES over every abtest/*.so (CIRUELA_AMD_LIB), chunk form
      for sh in ${SHAPES:-32768_16384 32768_32768 32768_49152 32768_65535 32768_98304 1048576_16384 1048576_32768 262144_65535}; do
        set -- ${sh/_/ }
        for lib in abtest/*.so; do
          CIRUELA_AMD_LIB=$PWD/$lib step "bs$1" 300 python bench.py --block-size $1 --blocks $2 --steps 5 \
            --warmup 1 --no-cpu-baseline > gpurun_out/shape.json 2> gpurun_out/shape.err
          echo "bs=$1 nblk=$2 $lib $(grep -o '"value": [0-9.]*' gpurun_out/shape.json)"
        done
      done ;;
    cli1)  # where a one-shot `ciruela-index sync` of config 1 spends its time
      python3 -c "import bench; bench.make_config1_tree('/tmp/cfg1_tree')"
      for r in 1 2 3; do
        step "hipinit$r" 60 ./build/hip_init_probe
      done
      for r in 1 2 3; do
        CIR_TRACE=1 step "cli$r" 60 python3 -c "import subprocess, sys, time; t = time.time(); \
rc = subprocess.call(['./bin/ciruela-index', 'sync', '--append', '/tmp/cfg1_tree:/bench'], \
stdout=subprocess.DEVNULL); print('cli wall %.3f s' % (time.time() - t), file=sys.stderr); sys.exit(rc)"
      done ;;
    cfg1)
      step cfg1 300 python bench.py --workload config1 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err
      cat gpurun_out/cfg1.json ;;
    cfg5)
      df -h /dev/shm /tmp | tee gpurun_out/df.txt
      free -g | tee -a gpurun_out/df.txt
      CIR_TRACE=${CIR_TRACE:-} step cfg5 1000 python bench.py --workload config5 --steps 3 --tree-gib "${TREE_GIB:-50}" \
        > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
      rm -rf /dev/shm/ciruela_bench_tree
      cat gpurun_out/cfg5.json ;;
    cfg5sweep)
      for t in ${THREADS:-8 16 32}; do
        CIR_SCAN_THREADS=$t CIR_TRACE=1 step "cfg5_t$t" 600 python bench.py --workload config5 --steps 2 \
          --tree-gib "${TREE_GIB:-8}" > gpurun_out/cfg5_t$t.json 2> gpurun_out/cfg5_t$t.err
        grep -o '"value": [0-9.]*\|"seconds_all": \[[0-9., ]*\]' gpurun_out/cfg5_t$t.json | head -2 | tr '\n' ' '
        grep "cir_scan dev 0 slot" gpurun_out/cfg5_t$t.err | awk '{h+=$7; n++} END {printf "  mean h2d %.2f ms over %d slots\n", h/n, n}'
        grep "cir_scan dev 0 batch" gpurun_out/cfg5_t$t.err | awk '{r+=$13; n++} END {printf "  mean read %.2f ms over %d batches\n", r/n, n}' 
      done
      rm -rf /dev/shm/ciruela_bench_tree ;;
    dist1)
      step dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 --force-dist \
        --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err
      cat gpurun_out/dist1.json ;;
    asmg)
      step asmg 300 ./build/asm_g_ubench > gpurun_out/asmg.log 2>&1
      cat gpurun_out/asmg.log ;;
    dvfs)
      step dvfs 300 ./build/dvfs_probe > gpurun_out/dvfs.log 2>&1
      cat gpurun_out/dvfs.log ;;
    quad)
      step quad 300 python tools/quad_probe.py > gpurun_out/quad.log 2>&1
      cat gpurun_out/quad.log ;;
    lat)
      step lat 300 ./build/lat_ubench > gpurun_out/lat.log 2>&1
      cat gpurun_out/lat.log ;;
    order)
      step order 300 ./build/order_ubench > gpurun_out/order.log 2>&1
      cat gpurun_out/order.log ;;
    ubench)
      step ubench 300 ./build/valu_ubench > gpurun_out/ubench.log 2>&1
      cat gpurun_out/ubench.log ;;
    pmcsq)  # one pass of SQ counters + GRBM over config 2 (k_chunks and the register-only k_compress_only)
      step pmcsq 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/pmcsq -o run -- python3 bench.py --steps 3 --warmup 1 \
        --no-cpu-baseline --no-secondary > gpurun_out/pmcsq.log 2>&1 ;;
    lanepmcab)  # dl32k as descriptors under one --pmc pass per abtest/*.so (clock + cycles)
      for lib in abtest/*.so; do
        n=$(basename "$lib" .so)
        CIRUELA_AMD_LIB=$PWD/$lib SWEEP_DESC=1 SWEEP_ONLY=32768:1048576 SWEEP_STEPS=3 step "lpmc_$n" 300 \
          rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
          SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv \
          -d "gpurun_out/lpmc_$n" -o run -- python3 tools/shape_sweep.py > "gpurun_out/lpmc_$n.log" 2>&1
      done ;;
    lanepmc)  # 1 M x 32 KiB as a chunk-form file (k_chunks, LDS-DMA) vs descriptors (k_lane_rest)
      for mode in 0 1; do
        SWEEP_DESC=$mode SWEEP_ONLY=32768:1048576 SWEEP_STEPS=10 step "lane_t$mode" 300 \
          python3 tools/shape_sweep.py > "gpurun_out/lane_t$mode.log" 2>&1
        cat "gpurun_out/lane_t$mode.log"
        SWEEP_DESC=$mode SWEEP_ONLY=32768:1048576 SWEEP_STEPS=3 step "lanepmc_$mode" 300 \
          rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM \
          --output-format csv -d "gpurun_out/lanepmc_$mode" -o run -- python3 tools/shape_sweep.py \
          > "gpurun_out/lanepmc_$mode.log" 2>&1
      done
      step counters 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 ;;
    xcdclk)  # is the shader clock per XCD? (tools/xcd_clock_probe.hip)
      step xcdclk 120 ./build/xcd_clock_probe > gpurun_out/xcdclk.log 2>&1
      cat gpurun_out/xcdclk.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
