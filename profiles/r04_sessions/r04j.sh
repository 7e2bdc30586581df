#!/bin/bash
# round 4: training GPU tests + train bench (3xf16 headline, f16 variant, fp32 reference)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
IFD_WGRAD_WS=1 timeout -k 10 120 python tools/diag/wgrad_time.py > $OUT/wgrad_ws1.txt 2>&1 || exit $?; echo "ws=1 $(grep x3=1 $OUT/wgrad_ws1.txt)"
IFD_PARITY_JSON=$OUT/parity_train.json timeout -k 10 900 python -u -m pytest tests/test_gpu_train_gn.py tests/test_gpu_wgrad.py tests/test_gpu_train_fuse.py tests/test_gpu_train.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/train_tests.txt 2>&1; rc=$?; echo "train tests rc=$rc"; tail -3 $OUT/train_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 2 --f16-steps 3 > $OUT/bench_train.json 2> $OUT/bench_train.err || exit $?
python -c "
import json
d=json.load(open('$OUT/bench_train.json'));print(d['value'],d['ms_per_step'],d.get('fp32_exact'),d.get('f16_reduced'))"
