#!/bin/bash
# round 4: the chunk interval's composition on the final build (timing-only ablations, garbage outputs):
# ab1 producers skip halo loads + LDS writes, ab2 producers skip prologue/split/LDS writes, ab4 consumers
# skip the 3x3 MFMAs; per-layer profile of the dominant layer for each
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for v in base ab1 ab2 ab4; do
  export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lpz_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lpz_$v.txt) | $(grep 'r256 128+0->128 skip0' $OUT/lpz_$v.txt | head -1 | cut -c60-)"
done
