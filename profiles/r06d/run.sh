#!/bin/bash
# round 6 session d: the training changes (wgrad_ws 8 x 8 chunks with 7 halo items per producer thread; the GNB dgrad
# epilogue's parameter loads in one round): every training test on the new in-tree library, then the training step
# interleaved against the round's previous library (tools/abl/libifd_base6.so, HEAD 4c16332) on this box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06d; mkdir -p $O
cd $R
IFD_PARITY_JSON=$O/parity_train.json timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_fuse.py \
  tests/test_gpu_wgrad.py tests/test_gpu_partial_tiles.py tests/test_gpu_train_gstat.py tests/test_gpu_train_gn.py \
  tests/test_gpu_train_attn.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/train_tests.txt 2>&1; rc=$?
echo "train tests rc=$rc: $(tail -1 $O/train_tests.txt)"; [ $rc -eq 0 ] || exit 1
T="--workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 --f16-steps 0"
for rep in 1 2; do
  for v in base6 new; do
    if [ $v = new ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 200 python bench.py $T > $O/train_${v}_$rep.json 2> $O/train_${v}_$rep.err || { echo "train $v failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/train_${v}_$rep.json'));print('$v $rep', d['value'], d['ms_per_step'])"
  done
done
unset IFD_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o trace --output-format csv -- python $R/bench.py $T > $O/trace_train.log 2>&1 || { echo "train trace failed"; exit 1; }
echo "trace ok"
