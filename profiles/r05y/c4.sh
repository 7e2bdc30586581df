#!/bin/bash
# round 5 session y2: the C4 path rehearsed on one device (2 ranks, global batch 17: shards of 9 and 8, a partial
# four-image tile on rank 0), device and parity noise
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y; mkdir -p $O
cd $R
for nz in device parity; do
  timeout -k 10 600 python bench.py --workload c4 --gpus 2 --global-batch 17 --noise $nz --steps 1 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/c4_$nz.json 2> $O/c4_$nz.err || { echo "c4 $nz failed"; tail -5 $O/c4_$nz.err; exit 1; }
  echo "stdout lines: $(wc -l < $O/c4_$nz.json)"
  python -c "import json;d=json.load(open('$O/c4_$nz.json'));print('c4 $nz', d['value'], d['n_gpus'], d['n_ranks'], d['config'].get('parallelism'))"
done
