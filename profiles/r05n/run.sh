#!/bin/bash
# round 5 session n: four-image 8x8 tiles at any batch (partial last tile) in the batch-invariant geometry:
# the split-kernel and invariance tests, parity-mode bench at B = 16 / 64 beside the device geometry, and the
# 2-rank rehearsal of the multi-GPU bench path on one device
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_x3.py tests/test_gpu_configs.py tests/test_gpu_full.py -k "partial or batch4 or shard or invariant or c4 or geometry" > $O/tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" $O/tests.txt | tail -14; [ $rc -eq 0 ] || exit 1
B="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0"
for b in 16 64; do
  timeout -k 10 400 python bench.py --noise parity --batch $b --steps 2 --warmup 1 $B > $O/bench_parity$b.json 2> $O/bench_parity$b.err || { echo "parity $b failed"; tail -3 $O/bench_parity$b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_parity$b.json'));print('parity$b', d['value'], d['ms_per_step'], d['config'].get('options'))"
  timeout -k 10 400 python bench.py --batch $b --steps 2 --warmup 1 $B > $O/bench_device$b.json 2> $O/bench_device$b.err || { echo "device $b failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_device$b.json'));print('device$b', d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 $B > $O/bench_gpus2_rehearsal.json 2> $O/bench_gpus2_rehearsal.err || { echo "rehearsal failed"; tail -5 $O/bench_gpus2_rehearsal.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_gpus2_rehearsal.json'));print('gpus2', d['value'], d['n_gpus'], d['config'].get('parallelism'))"
