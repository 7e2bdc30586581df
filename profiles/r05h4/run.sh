#!/bin/bash
# round 5 session h2: the output blocks' skip gradients added in the GroupNorm backward's dx pass (no separate
# accumulating channel copy). Training GPU tests; training bench; rocprof kernel trace of the training step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05h2}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py tests/test_gpu_train_gn.py tests/test_gpu_train_attn.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
      > $O/train_$rep.json 2> $O/train_$rep.err || { echo "train failed"; tail -5 $O/train_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/train_$rep.json'));print('rep $rep', d['value'], d['ms_per_step'], d['loss'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
