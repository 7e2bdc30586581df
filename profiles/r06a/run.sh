#!/bin/bash
# round 6 session a: the partial-tile fix (new tests, the round-5 repro asynchronously with partial tiles on in
# training), the drop-in loop with the lazy and the sync range guard, then the whole GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06a; mkdir -p $O
cd $R
IFD_PARITY_JSON=$O/parity_pt.json timeout -k 10 400 python -u -m pytest tests/test_gpu_partial_tiles.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/partial_tests.txt 2>&1; rc=$?
tail -4 $O/partial_tests.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/r05r/repro.py 2 3 > $O/repro_async.txt 2>&1; rc=$?
echo "repro rc=$rc"; grep -E "^=== step|^ok|Error" $O/repro_async.txt | tail -6; [ $rc -eq 0 ] || exit 1
B="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --train-steps 0"
for G in lazy sync; do
  IFD_GUARD=$G timeout -k 10 300 python bench.py --workload dropin --steps 2 --warmup 1 $B > $O/bench_dropin_$G.json 2> $O/bench_dropin_$G.err || { echo "dropin $G failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_dropin_$G.json'));print('dropin $G', d['value'], d.get('fused'))"
done
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -8
