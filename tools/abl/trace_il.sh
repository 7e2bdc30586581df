#!/bin/bash
# development: chunk-interval traces of the 256^2 skip layer (interleaved skip) for trace/ablation builds
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "$@"; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 150 python tools/x3_trace.py "r256 128+0->128 skip256" > gpurun_out/tr_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
done
