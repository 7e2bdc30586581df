#!/bin/bash
# round 6 session b: the default bench line (headline + fp32/f16 + the new training leg + cpu baseline), the
# drop-in guard test, a kernel trace and an MFMA-busy / clock PMC pass of the training step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b; mkdir -p $O
cd $R
IFD_PARITY_JSON=$O/parity_guard.json timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -k "range_guard" -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/guard_tests.txt 2>&1; rc=$?
tail -3 $O/guard_tests.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['roofline']['frac'], d.get('train'), d.get('fp32_exact',{}).get('value'), d.get('f16_reduced',{}).get('value'), d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
T="--workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o trace --output-format csv -- python $R/bench.py $T > $O/trace_train.log 2>&1 || { echo "train trace failed"; exit 1; }
echo "trace ok"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-include-regex "wgrad|conv_x3|gn_bwd|skip_x3" -d $O/pmc3_train -o pmc --output-format csv -- python $R/bench.py $T > $O/pmc3_train.log 2>&1 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
