#!/bin/bash
# round 6 session g: the GNB dgrad epilogue writes the GroupNorm's forward output for the next weight gradient
# (gnb_act): the training tests, then the training step with gnb_act on / off interleaved twice (same library)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g; mkdir -p $O
cd $R
IFD_PARITY_JSON=$O/parity_train.json timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_fuse.py \
  tests/test_gpu_wgrad.py tests/test_gpu_partial_tiles.py tests/test_gpu_train_gstat.py tests/test_gpu_train_gn.py \
  tests/test_gpu_train_attn.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/train_tests.txt 2>&1; rc=$?
echo "train tests rc=$rc: $(tail -1 $O/train_tests.txt)"; [ $rc -eq 0 ] || { grep -E "^E |Error" $O/train_tests.txt | head -20; exit 1; }
T="--workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 --f16-steps 0"
for rep in 1 2; do
  for v in 0 1; do
    IFD_TRAIN_GNB_ACT=$v timeout -k 10 200 python bench.py $T > $O/train_act${v}_$rep.json 2> $O/train_act${v}_$rep.err || { echo "train act=$v failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/train_act${v}_$rep.json'));print('gnb_act=$v $rep', d['value'], d['ms_per_step'])"
  done
done
