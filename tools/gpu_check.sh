#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout (exit other
# than 0 or 1) ends the script at once -- nothing further touches the GPU.
#   usage: tools/gpu_check.sh [steps...]
#   steps: smoke tests contract bench benchdrv benchnf bench5 benchbmf bench3 bench2gloo bench4gloo benchdist1 distcost benchsplit cpunproc
#          prof pmc pmc5 profbmf pmcbmf asm profasm pmcasm asmsweep ring capture matrix knobs
#          probe skew overlap spikes patterns asmprobe h2d diskdb idlerep keeprep tune tunebmf capturemt multi
#          benchbpl profbpl benchcmp ringq ringn drvx3 tunelay tunefs cpuspread cpuspread2 cputhreads sustained matrix4 pmc1
#          devleak devleak20 replay9090 debughunt hunt5 cpuwait gatherhunt churnrep
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
# device-ring holders (dada_db -g) left by a killed step exit after 15 idle minutes
export DADA_HOLDER_IDLE_S=900
OUT=gpurun_out
mkdir -p "$OUT"
STEPS=${*:-smoke tests bench prof}
# the libraries must be built from the sources in the snapshot (they are
# built here in the container, never on the box): refuse stale ones
if ! make -q -C paf-baseband2power_amd all >/dev/null 2>&1 || ! make -q -C oracle >/dev/null 2>&1; then
  echo "stale build: run make -C paf-baseband2power_amd all && make -C oracle before gpurun" | tee -a "$OUT/steps.log"
  exit 2
fi

run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name exit $rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with $rc" | tee -a "$OUT/steps.log"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1000 python3 -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread ;;
    contract) run pytest_contract 900 python3 -u -m pytest tests/test_gpu_bench_contract.py -x -v -rf \
                --timeout 800 --timeout-method thread ;;
    bench) run bench 600 python3 bench.py --steps 50 --warmup 5 ;;
    cpuspread) run cpu_spread 300 python3 tools/cpu_spread_probe.py 4 ;;
    cputhreads) run cpu_threads_a 300 python3 tools/cpu_spread_probe.py 4 spread2,spread2:14,spread2:15,spread2:12 &&
                run cpu_threads_b 300 python3 tools/cpu_spread_probe.py 4 spread2:15,spread2:14,spread2:12,spread2 ;;
    cpuspread2) run cpu_spread_a 300 python3 tools/cpu_spread_probe.py 4 spread,spread2,packed &&
                run cpu_spread_b 300 python3 tools/cpu_spread_probe.py 4 spread2,spread,packed ;;
    sustained) run bench_sustained 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --min-seconds 30 --cpu-seconds 0 ;;
    syncprobe) run sync_probe 300 python3 tools/sync_probe.py --regions 400 ;;
    benchdrv) run bench_drv 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchnf) run bench_nofuse 600 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-fuse ;;
    bench5) run bench_c5 600 python3 bench.py --config c5 --steps 30 --warmup 3 --cpu-seconds 0 ;;
    benchbmf) run bench_bmf 600 python3 bench.py --config bmf --steps 20 --warmup 3 --cpu-seconds 0 ;;
    bench2gloo) run bench_2gloo 600 python3 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo ;;
    bench4gloo) run bench_4gloo 600 python3 bench.py --gpus 4 --steps 10 --warmup 2 --dist-backend gloo ;;
    cpunproc) NCPU=$(python3 -c 'import os; print(os.cpu_count())')  # nproc follows OMP_NUM_THREADS
              run cpu_nproc 300 env OMP_NUM_THREADS=$NCPU OMP_PROC_BIND=close OMP_PLACES=threads \
              OMP_WAIT_POLICY=passive python3 oracle/cpu_baseline.py \
              '{"nbit":8,"nchan_chunk":256,"nsamp_df":1}' 6 20181105 &&
              run cpu_16 300 env OMP_NUM_THREADS=16 OMP_PROC_BIND=close OMP_PLACES=cores \
              OMP_WAIT_POLICY=active python3 oracle/cpu_baseline.py \
              '{"nbit":8,"nchan_chunk":256,"nsamp_df":1}' 6 20181105 ;;
    benchdist1) run bench_dist1 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
            --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 20 --warmup 2 \
            --cpu-seconds 0 --force-dist ;;
    distcost) for r in 1 2; do
                run dc_plain_r$r 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 &&
                run dc_dist_r$r 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                  --master-addr 127.0.0.1 --master-port $((29520 + r)) bench.py --steps 50 --warmup 5 \
                  --cpu-seconds 0 --force-dist || exit $?
              done ;;
    benchsplit) run bench_split1 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
            --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 20 --warmup 2 \
            --cpu-seconds 0 --force-dist --split time &&
          run bench_split2gloo 600 python3 bench.py --gpus 2 --steps 10 --warmup 2 \
            --dist-backend gloo --split time ;;
    benchbpl) for n in 2 4 8; do
                run bench_bpl$n 600 python3 bench.py --steps 48 --warmup 4 --cpu-seconds 0 --blocks-per-launch $n &&
                run bench_c5_bpl$n 600 python3 bench.py --config c5 --steps 24 --warmup 2 --cpu-seconds 0 \
                  --blocks-per-launch $n || exit $?
              done ;;
    benchcmp) for r in 1 2; do  # the driver's command, and the same with one block per launch
                run cmp_auto_r$r 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 &&
                run cmp_bpl1_r$r 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 \
                  --blocks-per-launch 1 || exit $?
              done ;;
    tunelay) # the two slowest layouts of the perf matrix
             run tune_i8_336 600 python3 tools/tune.py --case "int8 336ch" --quick &&
             run tune_tftfp88 600 python3 tools/tune.py --case "int16 BE TFTFP 8x8" --threads 128,256,512,1024 ;;
    tunefs) # frame-split workgroup sizes: TFTFP 8x8 and BMF, 5 rounds
             run tune_fs_tftfp88 600 python3 tools/tune.py --case "int16 BE TFTFP 8x8" --threads 256,512 --rounds 5 &&
             run tune_fs_bmf 600 python3 tools/tune.py --config bmf --threads 448,512 --rounds 5 ;;
    tuneil) # row interleave for multi-column int8 layouts
             run tune_il_336 600 python3 tools/tune.py --case "int8 336ch" --quick --rounds 5 &&
             run tune_il_tftfp32x8 600 python3 tools/tune.py --case "int8 TFTFP 32x8" --threads 256,512 --rounds 5 ;;
    drvx3) for r in 1 2 3; do  # the driver's command three times (no CPU leg)
             run drv_r$r 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 || exit $?
           done ;;
    ringq) # configs[1] blocks through the device ring: 2 blocks (one per launch) vs 8 (batched)
           run ring_q2 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 2 --blocks 400 &&
           run ring_q8 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 8 --blocks 400 &&
           run ring_q2b 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 2 --blocks 400 &&
           run ring_q8b 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 8 --blocks 400 ;;
    ringn) # one stage serving 2 sub-bands (-n 2, gathered) vs one, configs[1] blocks, one GPU
           run ring_n1 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 8 --blocks 200 &&
           run ring_n2 600 python3 tools/bench_ring.py --layout int8:256 --nbufs 8 --blocks 200 --nsub 2 ;;
    profbpl) run prof_bpl4 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bpl4" -o run \
            -- python3 bench.py --steps 48 --warmup 4 --cpu-seconds 0 --blocks-per-launch 4 ;;
    bench3) run bench_c3 600 python3 bench.py --config c3 --steps 4 --warmup 1 --cpu-seconds 0 ;;
    asm) run bench_assemble 600 python3 tools/bench_assemble.py --steps 10 --warmup 2 ;;
    profasm) run prof_asm 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_asm" -o run \
            -- python3 tools/bench_assemble.py --steps 10 --warmup 2 ;;
    asmsweep) for g in 4096 8192 16384; do
                run asm_g${g} 300 python3 tools/bench_assemble.py --grid $g \
                  --steps 10 --warmup 2 --order tm || exit $?
              done ;;
    ring) run bench_ring 600 python3 tools/bench_ring.py --blocks 200 &&
          run bench_ring_sync 600 python3 tools/bench_ring.py --blocks 200 --sync &&
          run bench_ring_host 600 python3 tools/bench_ring.py --blocks 20 --host ;;
    pmcasm) run pmc_fetch_asm 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_asm" -o run \
            -- python3 tools/bench_assemble.py --steps 4 --warmup 1 --order tm &&
         run pmc_write_asm 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_asm" -o run \
            -- python3 tools/bench_assemble.py --steps 4 --warmup 1 --order tm ;;
    matrix) run perf_matrix 600 python3 tools/perf_matrix.py --steps 20 ;;
    matrix4) run perf_matrix_m4 600 python3 tools/perf_matrix.py --steps 40 --multi 4 ;;
    multi) run multi_1 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "int8 64ch" &&
           run multi_8 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "int8 64ch" --multi 8 &&
           run multi_tf1 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "TFTFP 8x8" &&
           run multi_tf8 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "TFTFP 8x8" --multi 8 &&
           run multi_c2 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "int8 256ch" &&
           run multi_c2_4 300 python3 tools/perf_matrix.py --steps 40 --npol-out 1 --only "int8 256ch" --multi 4 ;;
    idlerep) run idle_rep0 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 &&
             run idle_rep3 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 \
               --sleep 3 &&
             run idle_rep0b 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 ;;
    keeprep) run keep_rep 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 --keep &&
             run free_rep 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 &&
             run keep_rep_b 300 python3 tools/perf_matrix.py --steps 20 --only "int8 256ch" --npol-out 1 --repeat 4 --keep ;;
    knobs) i=0
           for kv in '{"unroll":8}' '{"unroll":16}' '{"max_threads":448}' '{"max_threads":256}' \
                     '{"interleave":1}' '{"interleave":0}' '{"wg_per_cu":2}' '{"nontemporal":0}'; do
             i=$((i+1))
             run knob_$i 300 python3 tools/perf_matrix.py --tuning "$kv" --steps 20 --only "int8 256ch" --npol-out 2 &&
             run knob16_$i 300 python3 tools/perf_matrix.py --tuning "$kv" --steps 20 --only "int16 LE 256ch" --npol-out 1 || exit $?
           done ;;
    spikes) run overlap_dist 300 paf-baseband2power_amd/bin/overlap_probe 200 dist &&
            run prof_spikes 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_spikes" -o run \
              -- python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 ;;
    h2d) run h2d_probe 300 paf-baseband2power_amd/bin/h2d_probe ;;
    patterns) run read_patterns 300 paf-baseband2power_amd/bin/read_pattern_probe 40 ;;
    asmprobe) run asmprobe 300 paf-baseband2power_amd/bin/assemble_probe 10 ;;
    diskdb) run bench_diskdb 600 python3 tools/bench_diskdb.py --nint 8 --threads 16 ;;
    capture) run bench_capture 600 python3 tools/bench_capture.py ;;
    capturemt) run bench_capture_mt 900 python3 tools/bench_capture.py --rates 3200,4800,6400,8000 \
                 --rx-threads 1,0 --send-threads 3 ;;
    probe) run hbm_probe 300 paf-baseband2power_amd/bin/hbm_probe 1024 ;;
    skew) run skew_probe 300 paf-baseband2power_amd/bin/skew_probe ;;
    overlap) run overlap_probe 300 paf-baseband2power_amd/bin/overlap_probe 40 ;;
    tune) run tune_c2 600 python3 tools/tune.py --config c2 &&
          run tune_c5 600 python3 tools/tune.py --config c5 --quick &&
          run tune_bmf 600 python3 tools/tune.py --config bmf --quick ;;
    tunebmf) run tune_bmf2 600 python3 tools/tune.py --config bmf --threads 168,256,336,448,512 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
            -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    pmc) # 12 steps: every launch carries bench.py's default 4 blocks (c2); no one-per-launch leg
         run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
            -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify --bpl1-seconds 0 --secondary-seconds 0 &&
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
            -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify --bpl1-seconds 0 --secondary-seconds 0 ;;
    pmc1) # the one-block launch shape (MULTI=false) of configs[1]
         run pmc_fetch_bpl1 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_bpl1" -o run \
            -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify --blocks-per-launch 1 --secondary-seconds 0 &&
         run pmc_write_bpl1 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_bpl1" -o run \
            -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify --blocks-per-launch 1 --secondary-seconds 0 ;;
    pmc5) run pmc_fetch_c5 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c5" -o run \
            -- python3 bench.py --config c5 --steps 6 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify &&
         run pmc_write_c5 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c5" -o run \
            -- python3 bench.py --config c5 --steps 6 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify &&
         run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run \
            -- python3 bench.py --config c5 --steps 30 --warmup 3 --cpu-seconds 0 ;;
    profbmf) run prof_bmf 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bmf" -o run \
            -- python3 bench.py --config bmf --steps 20 --warmup 3 --cpu-seconds 0 ;;
    pmcbmf) run pmc_fetch_bmf 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_bmf" -o run \
            -- python3 bench.py --config bmf --steps 10 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify &&
         run pmc_write_bmf 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_bmf" -o run \
            -- python3 bench.py --config bmf --steps 10 --warmup 2 --cpu-seconds 0 --min-seconds 0 --no-verify ;;
    replay9090) # round 4's failing stage hunt, replayed after the device-ring ordering rule:
                # seed 9090 at scale 6, every GPU-resident ring written from the test process
                run replay9090 1100 env B2P_STAGE_WRITER=inproc B2P_HYPOTHESIS_SEED=9090 B2P_HYPOTHESIS_SCALE=6 \
                  python3 -u -m pytest tests/test_gpu_stage_random.py -v -rf --timeout 900 --timeout-method thread \
                  -k "layouts_rings_and_flags or gathered_subbands" --hypothesis-show-statistics ;;
    debughunt) # the host-staging property under the debug library, 1500 examples, seed 777
               run debug_staging_hunt 900 python3 -u tests/debug_build_checks.py staging 1500 777 ;;
    devleak20) run devring_leak20 900 python3 tools/devring_probe.py 20 use ;;
    hunt5) # round 5's host-memory rules at scale, fresh seeds: the ABI state machine (registration,
           # host-output finishes, unregister drains) and the host-staging property (release library)
           run hunt5_api 900 env B2P_HYPOTHESIS_SCALE=20 B2P_HYPOTHESIS_SEED=5151 python3 -u -m pytest \
             tests/test_gpu_api_model.py -v -s --timeout 800 --timeout-method thread --hypothesis-show-statistics &&
           run hunt5_staging 900 env B2P_HYPOTHESIS_SCALE=20 B2P_HYPOTHESIS_SEED=5152 python3 -u -m pytest \
             tests/test_gpu_random_layouts.py -k staging -v --timeout 800 --timeout-method thread \
             --hypothesis-show-statistics ;;
    gatherhunt) # the gathered C stage on GPU-resident rings (paf_diskdb writers), fresh seed, scale 5;
                # a failing stage's log is in the assertion (tests/test_gpu_device_ring.py _wait)
                run gather_hunt 900 env B2P_HYPOTHESIS_SEED=6161 B2P_HYPOTHESIS_SCALE=5 python3 -u -m pytest \
                  tests/test_gpu_stage_random.py -v -rf --timeout 800 --timeout-method thread \
                  -k "gathered_subbands and not inproc" --hypothesis-show-statistics ;;
    cpuwait) # the CPU baseline's thread count and OpenMP wait policy: spread and throttling
             run cpu_wait_a 300 python3 tools/cpu_spread_probe.py 5 \
               spread2:15:passive,spread2:15:default,spread2:15:active,spread2:14:passive,spread2:12:passive &&
             run cpu_wait_b 300 python3 tools/cpu_spread_probe.py 5 \
               spread2:12:passive,spread2:14:passive,spread2:15:active,spread2:15:default,spread2:15:passive ;;
    churnrep) # DESIGN.md item 1's candidate cause, tested: the recorded gathered case, each run right
              # after 6 device rings made, written from this process and destroyed back to back
              run case_churn 900 python3 -u tools/stage_case_repeat.py 30 churn=6 ;;
    devleak) # a few hundred device-ring create / write / destroy cycles in one process:
             # open fds and mapped size per ring
             run devring_leak 600 python3 tools/devring_probe.py 10 use ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps done" | tee -a "$OUT/steps.log"
