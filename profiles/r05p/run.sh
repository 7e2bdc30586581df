#!/bin/bash
# round 5 session p: four-image 8x8 tiles at every batch in the device geometry too (partial last tile): the split
# kernel tests at B = 1 / 3 / 4 / 5 / 16, and C1 (B = 1) in both geometries
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05p; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_x3.py tests/test_gpu_configs.py tests/test_gpu_full.py -k "batch or partial or shard or invariant or geometry or c1" > $O/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $O/tests.txt | tail -3; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.txt | head; exit 1; }
B="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0"
for nz in device parity; do
  timeout -k 10 300 python bench.py --batch 1 --ddim-steps 10 --eta 0.9 --noise $nz --steps 5 --warmup 2 $B > $O/bench_c1_$nz.json 2> $O/bench_c1_$nz.err || { echo "c1 $nz failed"; tail -3 $O/bench_c1_$nz.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c1_$nz.json'));print('c1 $nz', d['value'], d['ms_per_step'], d['unet_ms_per_eval'])"
done
timeout -k 10 400 python bench.py --batch 3 --steps 2 --warmup 1 $B > $O/bench_b3.json 2> $O/bench_b3.err || { echo "b3 failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_b3.json'));print('b3', d['value'], d['ms_per_step'], d['unet_ms_per_eval'])"
