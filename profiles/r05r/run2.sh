#!/bin/bash
# round 5 session r2: the padding-pixel address fix for partial four-image tiles (a spare slot's padding loads read
# below the tensor: faulted in the training conv path, whose tensors are separate allocations), then the wide 1x1
# weight gradient: conv repro cases, weight-gradient tests, training tests, sampler partial-tile tests, training
# bench twice and one traced step
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05r4}; mkdir -p $O
cd $R
for a in; do
  timeout -k 10 60 python -u profiles/r05r/repro2.py $a > $O/conv_${a// /_}.txt 2>&1 || { echo "FAILED at $a"; tail -2 $O/conv_${a// /_}.txt; exit 1; }
  tail -1 $O/conv_${a// /_}.txt
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wgrad.py > $O/wgrad_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $O/wgrad_tests.txt | tail -2; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py tests/test_gpu_train_gn.py tests/test_gpu_train_attn.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py tests/test_gpu_configs.py -k "train or gn or attn or gstat or block or c5 or split or addend" > $O/train_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $O/train_tests.txt | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/train_tests.txt | head -5; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x3.py tests/test_gpu_full.py -k "batch or partial or shard" > $O/x3_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $O/x3_tests.txt | tail -2; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
      > $O/train_$rep.json 2> $O/train_$rep.err || { echo "train failed"; tail -5 $O/train_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/train_$rep.json'));print('train rep $rep', d['value'], d['ms_per_step'], d['loss'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
