#!/bin/bash
# round 5 session g: timing ablations of the warp-specialised head (outputs garbage): 1 no consumer MFMAs,
# 2 no staging, 3 no halo loads, 4 no epilogue; hx0 = the round-2 head.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05g; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base hx0 hxa1 hxa2 hxa3 hxa4; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; tail -3 $O/lp_${v}_$rep.txt; exit 1; }
    echo "$v.$rep $(grep 'conv_head' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
