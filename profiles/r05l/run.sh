#!/bin/bash
# round 5 session l: batch-invariant geometry on a fixed reference batch of 16 (was 1): the invariance tests, and the
# parity-mode bench at B = 16 / 64 beside the device geometry
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_full.py -k "shard or invariant or arena or c4 or geometry" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit 1
for b in 16 64; do
  timeout -k 10 400 python bench.py --noise parity --batch $b --steps 2 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_parity$b.json 2> $O/bench_parity$b.err || { echo "parity $b failed"; tail -3 $O/bench_parity$b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_parity$b.json'));print('parity$b', d['value'], d['ms_per_step'], d['config'].get('options'))"
done
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_device64.json 2> $O/bench_device64.err || { echo "device64 failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_device64.json'));print('device64', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_device16.json 2> $O/bench_device16.err || { echo "device16 failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_device16.json'));print('device16', d['value'], d['ms_per_step'])"
