#!/bin/bash
# round 5 session i: skip_x3 timing ablations (outputs garbage): 1 no stores, 2 no MFMAs, 3 operand loads from one tile
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base ska1 ska2 ska3; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; tail -3 $O/lp_${v}_$rep.txt; exit 1; }
    echo "$v.$rep $(grep 'skip_x3 r256' $O/lp_${v}_$rep.txt | head -1 | cut -c60-) | $(grep 'skip_x3 r128 256' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
