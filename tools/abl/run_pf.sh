#!/bin/bash
# development: skip-layer timings of the prefetch-distance variants (tools/abl/libifd_pf*.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $R/gpurun_out/lp_$v.txt 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  echo "variant $v ok"
done
