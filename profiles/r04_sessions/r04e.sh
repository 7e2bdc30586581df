#!/bin/bash
# round 4: same-box layer-profile A/B of library variants (tools/abl/libifd_<v>.so; "new" = this tree)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
i=0
for v in ${VARIANTS:-new}; do
  i=$((i+1))
  if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python $R/tools/layer_prof.py ${LP_B:-16} 3xf16 > $OUT/lp_${i}_${v}.txt 2>&1 || { echo "layer prof $v failed"; exit 1; }
  echo "$v $(tail -1 $OUT/lp_${i}_${v}.txt) | $(grep 'r256 128+0->128 skip0' $OUT/lp_${i}_${v}.txt | head -1 | cut -c60-)"
done
