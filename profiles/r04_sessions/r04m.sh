#!/bin/bash
# round 4: full GPU tests + smoke + bench line of the current build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
PYTEST_X= bash $R/tools/gpu_tests.sh; rc=$?; echo "tests rc=$rc"; [ $rc = 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 500 python bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err || { echo "bench failed"; exit 1; }
python -c "
import json;d=json.load(open('$OUT/bench_final.json'));print(d['value'],d['unet_ms_per_eval'],d['roofline']['frac'],d['roofline']['traffic'],d['roofline'].get('traffic_source'),d.get('f16_reduced',{}).get('value'),d.get('fp32_exact',{}).get('value'))"
