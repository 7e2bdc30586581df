#!/bin/bash
# round 5 session g2: the head with 8 producer waves (in-tree) vs 4 (hxp4) vs the round-2 head (hx0): outputs,
# same-box layer profiles.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05g; mkdir -p $O
cd $R
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp2.txt 2>&1 || { echo "cmp base failed"; cat $O/cmp2.txt; exit 1; }
for v in hx0 hxp4; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/abl/cmp_lib.py $v --against base >> $O/cmp2.txt 2>&1 || { echo "cmp $v failed"; tail $O/cmp2.txt; exit 1; }
done
grep max-abs $O/cmp2.txt
for rep in 1 2; do
  for v in base hx0 hxp4; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp2_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; tail -3 $O/lp2_${v}_$rep.txt; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp2_${v}_$rep.txt) | $(grep 'conv_head' $O/lp2_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
