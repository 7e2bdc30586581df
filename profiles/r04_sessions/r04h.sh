#!/bin/bash
# round 4: warp-specialised wgrad variants (256^2, B = 32, 128 -> 128) + its tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for ws in 1 0; do IFD_WGRAD_WS=$ws timeout -k 10 120 python tools/diag/wgrad_time.py > $OUT/wgrad_ws$ws.txt 2>&1 || exit $?; echo "ws=$ws $(grep x3=1 $OUT/wgrad_ws$ws.txt)"; done
for v in ${VARIANTS-}; do IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/diag/wgrad_time.py > $OUT/wgrad_$v.txt 2>&1 || exit $?; echo "$v $(grep x3=1 $OUT/wgrad_$v.txt)"; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_train_fuse.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/wgrad_tests.txt 2>&1; echo "tests rc=$?"; tail -2 $OUT/wgrad_tests.txt
