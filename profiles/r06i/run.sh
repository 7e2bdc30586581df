#!/bin/bash
# round 6 session i: re-tune the handle option skip_sep (a ResBlock's 1x1 skip as its own skip_x3 launch at resolutions
# >= skip_sep, else as split-K skip chunks of conv2) on the final kernels: 64 (shipped), 128, 256 (never separate), 32
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06i; mkdir -p $O
cd $R
X="--steps 2 --warmup 1 --no-profile --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
for rep in 1 2; do
  for v in 64 128 512 32; do
    IFD_SKIP_SEP=$v timeout -k 10 200 python bench.py $X > $O/sep${v}_$rep.json 2> $O/sep${v}_$rep.err || { echo "sep $v failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/sep${v}_$rep.json'));print('skip_sep=$v $rep', d['value'], d['unet_ms_per_eval'])"
  done
done
