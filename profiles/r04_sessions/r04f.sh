#!/bin/bash
# round 4: training GPU tests and the training bench (3xf16 headline + fp32 + f16 variants)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
IFD_PARITY_JSON=$OUT/parity_train.json timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/train_tests.txt 2>&1; echo "train tests rc=$?"; tail -3 $OUT/train_tests.txt
timeout -k 10 600 python bench.py --workload train --batch 32 --steps 4 --warmup 1 --fp32-exact-steps 2 --f16-steps 3 > $OUT/bench_train.json 2> $OUT/bench_train.err; echo "train bench rc=$?"
python -c "import json;d=json.load(open('$OUT/bench_train.json'));print(d['value'],d['ms_per_step'],d.get('fp32_exact'),d.get('f16_reduced'))"
