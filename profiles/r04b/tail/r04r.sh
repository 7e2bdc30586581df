#!/bin/bash
# round 4: GN finalize / split-K statistics load batching — parity tests, then same-box timing vs the
# previous build (tools/abl/libifd_base.so)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_x3.py tests/test_gpu_full.py tests/test_gpu_blocks.py tests/test_gpu_f16.py tests/test_gpu_configs.py > $OUT/r_tests.txt 2>&1 || { tail -30 $OUT/r_tests.txt; exit 1; }
tail -2 $OUT/r_tests.txt
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/r_time.txt
  done
done
for v in base new; do
  if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lp_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lp_$v.txt) | $(grep -E 'groupnorm_stats' $OUT/lp_$v.txt | head -1 | cut -c60-)"
done
