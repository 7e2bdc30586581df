#!/bin/bash
# round 6 session h: the final library (after the gnb_act entry point; rerun as h2 after the empty-batch entry checks) - every GPU test, smoke, the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06h2; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['roofline']['frac'], d['train']['value'], d['fp32_exact']['value'], d['f16_reduced']['value'], d['cpu_baseline']['value'])"
