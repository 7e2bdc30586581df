#!/bin/bash
# GPU test pass on the box: one pytest process, per-test timeout, parity numbers to gpurun_out/parity.json.
# usage: tools/gpu_tests.sh [extra pytest args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
IFD_PARITY_JSON=$OUT/parity.json timeout -k 10 1000 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider "$@" > $OUT/gpu_tests.txt 2>&1
rc=$?
tail -5 $OUT/gpu_tests.txt
exit $rc
