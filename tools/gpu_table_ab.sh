# same-box A/B of two x3 contention tables through the whole model (per-mode throughput), alternated:
#   bash tools/gpu_table_ab.sh <table_a.json> <table_b.json> [slices, default dpx,qpx,cpx] [reps, default 2]
# (put both tables in the uploaded tree, e.g. under tools/; the shipped table is restored at the end)
set -u
A=$1; B=$2; SL=${3:-dpx,qpx,cpx}; REPS=${4:-2}
mkdir -p gpurun_out/tab
cp walkai_nos_amd/ops/x3_tuned.json gpurun_out/tab/shipped.json
for rep in $(seq 1 $REPS); do
  for t in a b; do
    if [ $t = a ]; then cp "$A" walkai_nos_amd/ops/x3_tuned.json; else cp "$B" walkai_nos_amd/ops/x3_tuned.json; fi
    timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --slices $SL --out gpurun_out/tab/modes_${t}_$rep.json > gpurun_out/tab/modes_${t}_$rep.log 2>&1 || { tail -20 gpurun_out/tab/modes_${t}_$rep.log; cp gpurun_out/tab/shipped.json walkai_nos_amd/ops/x3_tuned.json; exit 1; }
    grep mode gpurun_out/tab/modes_${t}_$rep.log | python -c "import sys,json; print('$t$rep', [(json.loads(l)['mode'][:3], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin])"
  done
done
cp gpurun_out/tab/shipped.json walkai_nos_amd/ops/x3_tuned.json
