#!/bin/bash
# round 4: nontemporal output stores in skip_x3 (sknt) vs the current build, same box, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for rep in 1 2 3; do
  for v in base sknt; do
    export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/sknt.txt
  done
done
