#!/bin/bash
# round 4: GroupNorm-on-load training (fuse_gn) + warp-specialised wgrad: tests, wgrad timing, train bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for ws in 0 1; do IFD_WGRAD_WS=$ws timeout -k 10 120 python tools/diag/wgrad_time.py > $OUT/wgrad_ws$ws.txt 2>&1 || exit $?; grep x3= $OUT/wgrad_ws$ws.txt; done
IFD_PARITY_JSON=$OUT/parity_train.json timeout -k 10 900 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_train_fuse.py tests/test_gpu_train.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/train_tests.txt 2>&1; rc=$?; echo "train tests rc=$rc"; tail -3 $OUT/train_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 --f16-steps 3 > $OUT/bench_train.json 2> $OUT/bench_train.err || exit $?
IFD_WGRAD_WS=0 timeout -k 10 300 python bench.py --workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 > $OUT/bench_train_ws0.json 2> $OUT/bench_train_ws0.err || exit $?
IFD_TRAIN_FUSE_GN=0 timeout -k 10 300 python bench.py --workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 0 > $OUT/bench_train_nofuse.json 2> $OUT/bench_train_nofuse.err || exit $?
python -c "
import json
for f in ('bench_train','bench_train_ws0','bench_train_nofuse'):
    d=json.load(open('$OUT/'+f+'.json'));print(f,d['value'],d['ms_per_step'],d.get('f16_reduced'))"
