#!/bin/bash
# round 6 final session: all GPU tests, smoke, the bench line + rocprof stats + PMC passes (tools/gpu_round.sh),
# the drop-in, parity, training and DDPM-1000 B=64 lines. Outputs under gpurun_out/r06z and gpurun_out/*_r06z.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
STEPS=5 bash tools/gpu_round.sh r06z || exit 1
B="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
timeout -k 10 400 python bench.py --workload dropin --steps 2 --warmup 1 $B > $O/bench_dropin.json 2> $O/bench_dropin.err || { echo "dropin failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_dropin.json'));print('dropin', d['value'], d.get('fused'))"
timeout -k 10 400 python bench.py --noise parity --steps 2 --warmup 1 $B > $O/bench_parity16.json 2> $O/bench_parity16.err || { echo "parity failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_parity16.json'));print('parity16', d['value'])"
timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 1 --f16-steps 1 > $O/bench_train.json 2> $O/bench_train.err || { echo "train failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_train.json'));print('train', d['value'], d['ms_per_step'], d.get('fp32_exact',{}).get('value'), d.get('f16_reduced',{}).get('value'))"
timeout -k 10 600 python -u bench.py --workload ddpm --batch 64 --steps 1 --warmup 0 $B > $O/bench_ddpm.json 2> $O/bench_ddpm.err || { echo "ddpm failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_ddpm.json'));print('ddpm', d['value'], d['ms_per_step'])"
