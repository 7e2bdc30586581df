#!/bin/bash
# round 5 session h: training step — GroupNorm-backward reduce + group means in one launch, slab + bias reductions in
# one launch, bias column sums always fused into the split weight-gradient kernels. Training GPU tests; same-box
# training bench A/B against tools/abl/libifd_gnr1.so (the previous reduce kernels).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py tests/test_gpu_train_gn.py tests/test_gpu_train_attn.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in base gnr1; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
        > $O/train_${v}_$rep.json 2> $O/train_${v}_$rep.err || { echo "train $v failed"; tail -5 $O/train_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/train_${v}_$rep.json'));print('$v rep $rep', d['value'], d['ms_per_step'], d['loss'])"
  done
done
unset IFD_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
