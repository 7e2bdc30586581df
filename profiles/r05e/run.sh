#!/bin/bash
# round 5 session e: the GroupNorm backward's pass 1 in the dgrad epilogue (training): GPU tests, smoke, the training
# step A/B (IFD_TRAIN_FUSE_GNB 0 / 1, interleaved), rocprof kernel stats of the fused training step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -8
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.txt
for rep in 1 2; do
  for f in 0 1; do
    IFD_TRAIN_FUSE_GNB=$f timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
        > $O/train_gnb${f}_$rep.json 2> $O/train_gnb${f}_$rep.err || { echo "train $f failed"; tail -5 $O/train_gnb${f}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/train_gnb${f}_$rep.json'));print('gnb=$f rep $rep', d['value'], d['ms_per_step'], d['loss'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
exit $rc
