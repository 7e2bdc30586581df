#!/bin/bash
# round 4: tree-reduced epilogue statistics (tree) vs the previous build (base): parity, same-box
# interleaved timing, dominant-layer profile, and the unit-transition trace of the new build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
IFD_LIB_PATH=$R/tools/abl/libifd_tree.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x3.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py tests/test_gpu_full.py > $OUT/tree_tests.txt 2>&1
rc=$?; tail -2 $OUT/tree_tests.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2 3; do
  for v in base tree; do
    export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so
    r=$(QT_N=20 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/tree.txt
  done
done
for v in base tree; do
  export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so
  timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $OUT/lpt_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/lpt_$v.txt) | $(grep 'r256 128+0->128 skip0' $OUT/lpt_$v.txt | head -1 | cut -c60-)"
done
IFD_LIB_PATH=$R/tools/abl/libifd_trace.so timeout -k 10 200 python tools/x3_trace.py "r256 128+0->128" > $OUT/x3trace_tree.txt 2>&1 || exit 1
grep -E "interval|epilogue" $OUT/x3trace_tree.txt
