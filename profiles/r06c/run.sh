#!/bin/bash
# round 6 session c: wgrad_ws_kernel chunk shape (WS_WC = 32 shipped, 16, 8: 64-pixel chunks of 2 x 32, 4 x 16, 8 x 8
# pixels, X halo 136 / 108 / 100 pixels). Correctness of each variant (the wgrad tests), then the training step
# interleaved twice per variant on this box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c; mkdir -p $O
cd $R
for v in wc8 wc16; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_train_fuse.py \
    -k "wgrad" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$v.txt 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 $O/tests_$v.txt)"; [ $rc -eq 0 ] || exit 1
done
T="--workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 --f16-steps 0"
for rep in 1 2; do
  for v in base wc8 wc16; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 200 python bench.py $T > $O/train_${v}_$rep.json 2> $O/train_${v}_$rep.err || { echo "train $v failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/train_${v}_$rep.json'));print('$v $rep', d['value'], d['ms_per_step'])"
  done
done
