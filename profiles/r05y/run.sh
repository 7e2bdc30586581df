#!/bin/bash
# round 5 session y: the whole GPU suite and smoke on the final library (after the training 1x1 change)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt $O/; echo "tests rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.txt | tail -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
