#!/bin/bash
# development: per-layer timings of the X3W_ABLATE variants (tools/abl/libifd_w*.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-0 1 2 3 4 5}; do
  if [ $v = 0 ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_w$v.so; fi
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $R/gpurun_out/ablw$v.txt 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  echo "variant $v ok"
done
