#!/bin/bash
# round 6 session k: per-layer profile of one UNet eval on the final library (B = 16, 3xf16), twice
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06k; mkdir -p $O
cd $R
for rep in 1 2; do
  timeout -k 10 180 python tools/layer_prof.py 16 3xf16 > $O/lp_$rep.txt 2>&1 || { echo "layer_prof failed"; tail -3 $O/lp_$rep.txt; exit 1; }
  tail -1 $O/lp_$rep.txt
done
