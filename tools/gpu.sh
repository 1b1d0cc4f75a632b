#!/bin/bash
# The one GPU runner for gpurun boxes: named steps, each under its own time limit; a fault, an
# abort or a timeout ends the run there (no retries). Results land under gpurun_out/.
#
#   bash tools/gpu.sh <step> [<step> ...]
#
# steps:
#   tests              pytest -m gpu (in one process)
#   test_k             pytest -m gpu -k "$NOS_TEST_K"
#   smoke              __graft_entry__.smoke()
#   bench              bench.py as the driver runs it (--gpus 1 --steps 20 --warmup 5)
#   bench_ranks        the driver's N > 1 launch rehearsed on the one GPU: NOS_RANKS ranks (default 2) over gloo
#   bench_torch        bench.py on the PyTorch (hipBLASLt) backend, for comparison
#   seeds              the bench window over churn seeds 1-5 and 1234 (NOS_SEEDS overrides)
#   operator           tools/operator_gpu_report.py: device map, commit barrier, probes
#   pod_start          tools/pod_start_probe.py: a pod process's boot phase by phase (1/8-GPU slice)
#   multiproc          tools/multiproc.py: pods as separate processes (sharing table, config 3)
#   curve              tools/sharing_curve.py: thread-emulated 1/3/5/7 sharing curve
#   prof               rocprofv3 kernel trace + stats of a short bench run
#   mprof              rocprofv3 kernel stats of whole inferences on one slice (NOS_SLICE, default spx)
#   pmc_op             PMC passes over one op (NOS_OP, NOS_SLICE), counters in their own runs
#   pmc_modes          L2 counters of a partition mode with all partitions busy (NOS_MODE, NOS_PARTS)
#   kbench             tools/kbench.py per-op / per-mode microbenchmarks (NOS_KBENCH_ARGS)
#   bench_runs         bench.py once per NOS_BENCH_RUNS entry ("<tag>:<arg>,<arg> ..."), e.g. layouts / seeds
#   bench_long         bench.py over NOS_STEPS quanta (default 100) for a longer window
#   fair               tools/gpu_fair.sh: memory-only fairness as processes (NOS_FAIR_ONLY, NOS_FAIR_VARIANTS)
#   fair_probe         tools/fair_probe.py: per-pod rates, amd-smi CU occupancy, KFD queues (NOS_FAIR_PODS)
#   replay             tools/model_replay.py + replay_stats kernel traces per slice (NOS_SLICES, default "dpx cpx")
#   procs_cap          tools/multiproc.py at 8-12 memory-only pods + the KFD queue properties
#   cu_guard           the CU-mask bypass guard test on real amd-smi (gpurun_out/cu_guard_samples.json)
#   attn_proj          tools/attn_proj_probe.py: fused merge+projection+LayerNorm vs the unfused launches
#   pmc_attn_proj      PMC passes over the fused kernel (NOS_ABLATE = its timing-only ablation mask)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/gpu_sh.log"

step() {  # step <name> <timeout> <cmd...>: run, log, stop the run on fault/abort/timeout
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/gpu_sh.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/gpu_sh.log"
  tail -n 4 "$OUT/$name.log" | tee -a "$OUT/gpu_sh.log"
  if [ $rc -ne 0 ]; then
    echo "stopping: $name ended with rc=$rc" | tee -a "$OUT/gpu_sh.log"
    exit $rc
  fi
}

pmc() {  # pmc <dir> <tag> <program...> -- <counters>: one counter pass, kernel trace only
  local dir=$1 tag=$2; shift 2
  local prog=()
  while [ "$1" != "--" ]; do prog+=("$1"); shift; done
  shift
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$dir" -o "$tag" -- \
    "${prog[@]}") > "$dir/$tag.log" 2>&1
}

for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread ;;
    test_k) step "test_${NOS_TEST_K:-x}" 600 python -u -m pytest tests -m gpu -x -v -rfP --timeout 300 \
              --timeout-method thread -k "${NOS_TEST_K:-x}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 --out "$OUT/bench.json" ;;
    bench_ranks) step "bench_${NOS_RANKS:-2}rank" 900 env NOS_BENCH_DIST_BACKEND=gloo python -m torch.distributed.run \
                   --nnodes=1 --nproc-per-node "${NOS_RANKS:-2}" --master-addr 127.0.0.1 --master-port 29517 bench.py \
                   --gpus "${NOS_RANKS:-2}" --steps 20 --warmup 5 --no-density ;;
    bench_torch) step bench_torch 600 python bench.py --steps 20 --warmup 5 --backend torch --out "$OUT/bench_torch.json" ;;
    seeds)
      mkdir -p "$OUT/seeds"
      for seed in ${NOS_SEEDS:-1 2 3 4 5 1234}; do
        step "seed_$seed" 300 python bench.py --no-density --seed "$seed" --out "$OUT/seeds/b_$seed.json"
      done ;;
    operator) step operator 600 python tools/operator_gpu_report.py --out "$OUT/operator.json" ;;
    pod_start) step pod_start 400 python tools/pod_start_probe.py --runs 3 --out "$OUT/pod_start_probe.json" ;;
    multiproc) step multiproc 900 python tools/multiproc.py --out "$OUT/multiproc.json" ${NOS_MP_ARGS:-} ;;
    curve) step sharing_curve 500 python tools/sharing_curve.py --seconds 4 --out "$OUT/sharing_curve.json" ;;
    prof)
      mkdir -p "$OUT/prof"
      step rocprof_bench 600 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d '$OUT/prof' -o bench \
        --output-format csv -- python3 '$ROOT/bench.py' --steps 6 --warmup 1 --no-density" ;;
    mprof)
      mkdir -p "$OUT/mprof"
      step mprof 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d '$OUT/mprof' -o model \
        -- python3 '$ROOT/tools/kbench.py' --only model --slices ${NOS_SLICE:-spx} --iters 8 --out '$OUT/mprof/kb.json'" ;;
    pmc_op)
      D="$OUT/pmc_${NOS_OP:-attn_x3}_${NOS_SLICE:-spx}"; mkdir -p "$D"
      P=(python3 "$ROOT/tools/kdrive.py" --op "${NOS_OP:-attn_x3}" --slice "${NOS_SLICE:-spx}")
      pmc "$D" p1 "${P[@]}" -- SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
          SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU && \
      pmc "$D" p2 "${P[@]}" -- SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE \
          GRBM_GUI_ACTIVE GRBM_COUNT && \
      pmc "$D" p3 "${P[@]}" -- TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
      pmc "$D" p4 "${P[@]}" -- TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
      rc=$?; echo "pmc_op rc=$rc" | tee -a "$OUT/gpu_sh.log"; [ $rc -eq 0 ] || exit $rc ;;
    pmc_modes)
      D="$OUT/pmc_modes_${NOS_MODE:-cpx}_${NOS_PARTS:-8}"; mkdir -p "$D"
      pmc "$D" p python3 "$ROOT/tools/kbench.py" --only modes --slices "${NOS_MODE:-cpx}" --partitions "${NOS_PARTS:-8}" \
          --out "$D/kb.json" -- TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum
      rc=$?; echo "pmc_modes rc=$rc" | tee -a "$OUT/gpu_sh.log"; [ $rc -eq 0 ] || exit $rc ;;
    attn_proj) step attn_proj 300 python tools/attn_proj_probe.py --iters 400 --out "$OUT/attn_proj.json" ;;
    pmc_attn_proj)
      D="$OUT/pmc_attn_proj"; mkdir -p "$D"
      P=(python3 "$ROOT/tools/attn_proj_probe.py" --iters 40 --ablate "${NOS_ABLATE:-0}" --fused-only)
      pmc "$D" p1 "${P[@]}" -- SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
          SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
      pmc "$D" p2 "${P[@]}" -- SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
          SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT && \
      pmc "$D" p3 "${P[@]}" -- TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
      pmc "$D" p4 "${P[@]}" -- TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
      rc=$?; echo "pmc_attn_proj rc=$rc" | tee -a "$OUT/gpu_sh.log"; [ $rc -eq 0 ] || exit $rc ;;
    kbench) step kbench 600 python tools/kbench.py ${NOS_KBENCH_ARGS:-} --out "$OUT/kbench.json" ;;
    bench_runs)
      for spec in ${NOS_BENCH_RUNS:-slices_1234:--layout=slices partitions_1234:--layout=partitions}; do
        tag=${spec%%:*}; args=${spec#*:}
        step "bench_$tag" 400 python -u bench.py ${args//,/ } --out "$OUT/bench_$tag.json"
      done ;;
    bench_long) step "bench_${NOS_STEPS:-100}q" 900 python -u bench.py --steps "${NOS_STEPS:-100}" --warmup 5 \
                  --out "$OUT/bench_${NOS_STEPS:-100}q.json" ;;
    fair) step fair 1100 bash tools/gpu_fair.sh ;;
    fair_probe) step fair_probe 900 python -u tools/fair_probe.py --pods "${NOS_FAIR_PODS:-5,7,8}" \
                  --reps "${NOS_FAIR_REPS:-2}" ${NOS_FAIR_ARGS:-} --out "$OUT/fair_probe.json" ;;
    replay)
      mkdir -p "$OUT/replay"
      for sl in ${NOS_SLICES:-dpx cpx}; do
        step "replay_$sl" 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --output-format csv -d '$OUT/replay' -o $sl \
          -- python3 '$ROOT/tools/model_replay.py' --slice $sl --replays 20"
        f=$(find "$OUT/replay" -name "${sl}_kernel_trace.csv" | sort | tail -1)
        step "replay_stats_$sl" 120 python tools/replay_stats.py "$f" --replays 20
      done ;;
    procs_cap)
      step procs_cap 700 python -u tools/multiproc.py --seconds 8 --only shared_8,shared_9,shared_10,shared_12 \
        --out "$OUT/procs_cap.json"
      for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do
        grep -H -E "simd_count|max_waves|num_cp_queues|num_xcc|cp_queue|vmid" "$f" || true
      done > "$OUT/kfd_props.txt" 2>&1 ;;
    cu_guard) step cu_guard 300 python -u -m pytest tests/test_gpu_native.py -x -v -rs -s --timeout 240 \
                --timeout-method thread -k cu_guard ;;
    *) echo "unknown step $s" | tee -a "$OUT/gpu_sh.log"; exit 2 ;;
  esac
done
echo "gpu.sh done" | tee -a "$OUT/gpu_sh.log"
