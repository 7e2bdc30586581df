#!/bin/bash
# round 4 measurement session: GPU tests, bench line, rocprofv3 kernel stats, PMC passes (tools/gpu_round.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
TAG=${1:-r04}
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  PYTEST_X= bash $R/tools/gpu_tests.sh; rc=$?; echo "tests rc=$rc"; [ $rc = 0 ] || exit 1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
  tail -1 $OUT/smoke.txt
fi
STEPS=${STEPS:-3} bash $R/tools/gpu_round.sh $TAG || exit 1
python $R/tools/pmc_summary.py $OUT $TAG > $OUT/pmc_summary_$TAG.json && echo "pmc summary ok"
