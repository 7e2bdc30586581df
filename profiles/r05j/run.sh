#!/bin/bash
# round 5 session j (mid-round full check): all GPU tests, smoke, the bench line + rocprof stats + PMC passes
# (tools/gpu_round.sh), the drop-in and training lines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
STEPS=5 bash tools/gpu_round.sh r05j || exit 1
timeout -k 10 400 python bench.py --workload dropin --steps 2 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_dropin.json 2> $O/bench_dropin.err || { echo "dropin failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_dropin.json'));print('dropin', d['value'], d.get('fused'))"
timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_train.json 2> $O/bench_train.err || { echo "train failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
