#!/bin/bash
# round 4: same-box layer-profile A/B (round-3 library vs this tree) + chunk-interval trace of the 8-chunk layer
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
IFD_LIB_PATH=$R/tools/abl/libifd_trace.so timeout -k 10 150 python tools/x3_trace.py "r256 128+0->128 skip0" > $OUT/tr8.txt 2>&1 || { echo "trace failed"; exit 1; }
grep -v amdgpu $OUT/tr8.txt | head -3; tail -1 $OUT/tr8.txt
i=0
for v in ${VARIANTS:-r03 new r03 new}; do
  i=$((i+1))
  if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $OUT/lp_${i}_${v}.txt 2>&1 || { echo "layer prof $v failed"; exit 1; }
  echo "$v $(tail -1 $OUT/lp_${i}_${v}.txt)"
done
