#!/bin/bash
# round 4: skip_sep threshold A/B (interleaved, same box)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for rep in 1 2; do
  for sep in ${SEPS:-64 0 128 256}; do
    r=$(IFD_SKIP_SEP=$sep QT_N=30 timeout -k 10 120 python tools/quick_time.py 16 3xf16 2>/dev/null | tail -1) || exit 1
    echo "sep=$sep $r" | tee -a $OUT/skip_sep.txt
  done
done
