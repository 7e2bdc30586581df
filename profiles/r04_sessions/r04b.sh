#!/bin/bash
# round 4: same-box A/B layer profiles (round-3 library, variants, this tree), GPU tests, bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
i=0
for v in ${VARIANTS:-r03 resil0 new r03 resil0 new}; do
  i=$((i+1))
  if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $OUT/lp_${i}_${v}.txt 2>&1 || { echo "layer prof $v failed"; exit 1; }
  echo "$v $(tail -1 $OUT/lp_${i}_${v}.txt)"
done
unset IFD_LIB_PATH
[ "${SKIP_TESTS:-0}" = 1 ] || { PYTEST_X= bash $R/tools/gpu_tests.sh; echo "tests rc=$?"; }
timeout -k 10 300 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['unet_ms_per_eval'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"
