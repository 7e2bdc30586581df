#!/bin/bash
# development: skip_x3 tuning variants (tools/abl/libifd_k*.so): per-layer timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-0 a b c}; do
  if [ $v = 0 ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_k$v.so; fi
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $R/gpurun_out/ablk$v.txt 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  echo "variant $v ok"
done
