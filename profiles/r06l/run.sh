#!/bin/bash
# round 6 session l: the C4 per-rank shape (64 images per GPU, DDIM-100 cosine, eta 0.75) on the final library, device
# and parity (batch-invariant geometry) noise: the per-GPU rate an 8-GPU C4 run would multiply
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l; mkdir -p $O
cd $R
X="--batch 64 --steps 1 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
for nz in device parity; do
  timeout -k 10 400 python bench.py $X --noise $nz > $O/b64_$nz.json 2> $O/b64_$nz.err || { echo "b64 $nz failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/b64_$nz.json'));print('B=64 $nz', d['value'], d['unet_ms_per_eval'], d['roofline']['frac'])"
done
