#!/bin/bash
# round 5 session i2: skip_x3 with transposed dwordx4 stores (in-tree) vs dword stores (skw0): outputs, layer profiles
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i; mkdir -p $O
cd $R
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp2.txt 2>&1 || { echo "cmp base failed"; cat $O/cmp2.txt; exit 1; }
IFD_LIB_PATH=$R/tools/abl/libifd_skw0.so timeout -k 10 120 python tools/abl/cmp_lib.py skw0 --against base >> $O/cmp2.txt 2>&1 || { echo "cmp failed"; tail $O/cmp2.txt; exit 1; }
grep max-abs $O/cmp2.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "skip or x3_matches or c2_ddim100" tests/ > $O/tests2.txt 2>&1; rc=$?
tail -2 $O/tests2.txt; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in base skw0; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp2_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; tail -3 $O/lp2_${v}_$rep.txt; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp2_${v}_$rep.txt) | $(grep 'skip_x3 r256' $O/lp2_${v}_$rep.txt | head -1 | cut -c60-) | $(grep 'skip_x3 r128 256' $O/lp2_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
