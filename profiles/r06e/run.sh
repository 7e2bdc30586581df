#!/bin/bash
# round 6 session e: where the 3x3 split weight gradient's time goes (timing-only WS_ABL builds, outputs garbage):
# 1 producers idle after the first chunk (consumer-bound time), 2 consumers without MFMAs (producer-bound time),
# 5 producers without LDS writes; the in-tree build between them, twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06e; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base wsabl1 wsabl2 wsabl5; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/diag/wgrad_abl.py > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "$v failed"; tail -3 $O/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $O/${v}_$rep.json)"
  done
done
