#!/bin/bash
# round 6 session f: the final library's C4 path rehearsed on one device (2 ranks over gloo, global batch 17: shards of
# 9 and 8, a partial four-image tile on rank 0), device and parity noise; and C1 (B = 1, 10-step DDIM cosine, eta 0.9)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f; mkdir -p $O
cd $R
X="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
for nz in device parity; do
  timeout -k 10 600 python bench.py --workload c4 --gpus 2 --global-batch 17 --noise $nz --steps 1 --warmup 1 $X > $O/c4_$nz.json 2> $O/c4_$nz.err || { echo "c4 $nz failed"; tail -5 $O/c4_$nz.err; exit 1; }
  echo "stdout lines: $(wc -l < $O/c4_$nz.json)"
  python -c "import json;d=json.load(open('$O/c4_$nz.json'));print('c4 $nz', d['value'], d['n_gpus'], d['n_ranks'], d['config'].get('parallelism'))"
done
timeout -k 10 300 python bench.py --batch 1 --ddim-steps 10 --eta 0.9 --steps 5 --warmup 1 $X > $O/c1.json 2> $O/c1.err || { echo "c1 failed"; exit 1; }
python -c "import json;d=json.load(open('$O/c1.json'));print('c1', d['value'], d['ms_per_step'], d['unet_ms_per_eval'])"
