# headline bench over several churn seeds (which pods happen to be in the timed window)
set -u
mkdir -p gpurun_out/r2aq
for seed in 1 2 3 4 5 1234; do
  timeout -k 10 600 python bench.py --seed $seed --no-density > gpurun_out/r2aq/seed_$seed.json 2> gpurun_out/r2aq/seed_$seed.err || exit 1
done
