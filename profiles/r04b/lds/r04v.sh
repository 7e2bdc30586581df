#!/bin/bash
# round 4: cost of the residual prefetch — a17 (no residual loads, the epilogue adds zeros; timing only)
# vs the shipped build, same box, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in base a17; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/a17.txt
  done
done
for v in base a17; do
  if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lp_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lp_$v.txt)"; grep -E "r256 128\+0->128 skip0|r256 128\+128->128 skip0|r128 128\+0->128 skip0" $OUT/lp_$v.txt | cut -c1-110
done
