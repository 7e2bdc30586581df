#!/bin/bash
# round 5 session a: the dominant conv's epilogue variants, same box. Outputs under gpurun_out/r05a/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a; mkdir -p $O
cd $R
# outputs: every real variant against the in-tree build (bit-equal expected except e4, the tree order)
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp.txt 2>&1 || { echo "cmp base failed"; cat $O/cmp.txt; exit 1; }
for v in head e1 e2 e3 e4; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/abl/cmp_lib.py $v --against base >> $O/cmp.txt 2>&1 || { echo "cmp $v failed"; exit 1; }
done
cat $O/cmp.txt | grep max-abs
# layer profiles, two interleaved rounds
for rep in 1 2; do
  for v in base head e1 e2 e3 e4 ab13 ab14 ab15 ab17; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp_${v}_$rep.txt) | $(grep 'r256 128+0->128 skip0 xf0' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
unset IFD_LIB_PATH
for v in tr0 tr3; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/x3_trace.py 'r256 128+0->128 skip0 xf0' > $O/trace_$v.txt 2>&1 || { echo "trace $v failed"; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/trace_$v.txt
done
