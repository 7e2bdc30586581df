#!/bin/bash
# round 5 session f: warp-specialised head (in-tree) vs the round-2 head (tools/abl/libifd_hx0.so): outputs
# bit for bit, head GPU tests, same-box layer profiles (two interleaved repetitions).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f; mkdir -p $O
cd $R
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp.txt 2>&1 || { echo "cmp base failed"; cat $O/cmp.txt; exit 1; }
IFD_LIB_PATH=$R/tools/abl/libifd_hx0.so timeout -k 10 120 python tools/abl/cmp_lib.py hx0 --against base >> $O/cmp.txt 2>&1 || { echo "cmp hx0 failed"; tail $O/cmp.txt; exit 1; }
grep max-abs $O/cmp.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "head or c2_ddim100 or c3_ddpm or dropin or x3_matches or gpu_parity" tests/ > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in base hx0; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp_${v}_$rep.txt) | $(grep 'conv_head' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
