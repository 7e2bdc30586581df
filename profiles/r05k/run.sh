#!/bin/bash
# round 5: batched weight packing A/B (IFD_TRAIN_PACK_BATCH 1 / 0), training bench, interleaved; trace of the batched
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for b in 1 0; do
    IFD_TRAIN_PACK_BATCH=$b timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
        > $O/train_b${b}_$rep.json 2> $O/train_b${b}_$rep.err || { echo "train failed"; tail -5 $O/train_b${b}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/train_b${b}_$rep.json'));print('batch=$b rep $rep', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
