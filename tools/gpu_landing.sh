# landing-CU partition emulation: census test, per-mode throughput (landing vs spread), bench A/B
set -u
mkdir -p gpurun_out/landing
timeout -k 10 300 python -u -m pytest tests/test_gpu_pin.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/landing/pytest_pin.log 2>&1 || { tail -30 gpurun_out/landing/pytest_pin.log; exit 1; }
tail -3 gpurun_out/landing/pytest_pin.log
for em in landing spread; do
  timeout -k 10 400 python tools/kbench.py --only modes --emulation $em --out gpurun_out/landing/modes_$em.json > gpurun_out/landing/modes_$em.log 2>&1 || { tail -20 gpurun_out/landing/modes_$em.log; exit 1; }
  grep mode gpurun_out/landing/modes_$em.log | python -c "import sys,json; [print('$em', json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
done
for em in landing spread; do
  timeout -k 10 300 python bench.py --emulation $em --out gpurun_out/landing/bench_$em.json > /dev/null 2> gpurun_out/landing/bench_$em.err || { tail -30 gpurun_out/landing/bench_$em.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/landing/bench_$em.json')); print('bench $em', d['value'], d['density'])"
done
