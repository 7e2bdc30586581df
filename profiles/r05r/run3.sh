#!/bin/bash
# round 5 session x: the training step's 1x1 convs at >= 64^2 on the dedicated split 1x1 kernel (ifd_tr_conv1x1_x3):
# its tests, the training tests, the training bench twice and one traced step
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05x}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train_fuse.py -k conv1x1 > $O/c11_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" $O/c11_tests.txt | tail -6; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/c11_tests.txt | head -5; exit 1; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py tests/test_gpu_train_gn.py tests/test_gpu_train_attn.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py tests/test_gpu_configs.py tests/test_gpu_wgrad.py -k "train or gn or attn or gstat or block or c5 or split or addend or wgrad" > $O/train_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $O/train_tests.txt | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/train_tests.txt | head -5; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 1 \
      > $O/train_$rep.json 2> $O/train_$rep.err || { echo "train failed"; tail -5 $O/train_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/train_$rep.json'));print('train rep $rep', d['value'], d['ms_per_step'], d['loss'], d.get('f16_reduced',{}).get('value'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
