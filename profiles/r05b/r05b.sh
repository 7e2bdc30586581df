#!/bin/bash
# round 5 session b: deferred output stores (X3_DEFER=4 in-tree; d0 = off, d2 = two phases) + the lazy guard:
# GPU tests, smoke, same-box layer A/B, the unit-transition trace, bench lines (headline, drop-in, parity B16/B64).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/ 2>/dev/null; echo "tests rc=$rc"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp.txt 2>&1 || { echo "cmp base failed"; exit 1; }
for v in d0 d2; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/abl/cmp_lib.py $v --against base >> $O/cmp.txt 2>&1 || { echo "cmp $v failed"; exit 1; }
done
grep max-abs $O/cmp.txt
for rep in 1 2; do
  for v in base d0 d2; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp_${v}_$rep.txt) | $(grep 'r256 128+0->128 skip0 ' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
unset IFD_LIB_PATH
IFD_LIB_PATH=$R/tools/abl/libifd_trd4.so timeout -k 10 120 python tools/x3_trace.py 'r256 128+0->128 skip0 xf0' > $O/trace_d4.txt 2>&1 || { echo "trace failed"; exit 1; }
grep -v amdgpu.ids $O/trace_d4.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d['unet_ms_per_eval'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('fp32_exact',{}).get('value'),d.get('f16_reduced',{}).get('value'),d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --workload dropin --cpu-baseline-seconds 0 > $O/bench_dropin.json 2> $O/bench_dropin.err || { echo "dropin failed"; tail -5 $O/bench_dropin.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_dropin.json'));print('dropin',d['value'],d['fused'])"
timeout -k 10 300 python bench.py --noise parity --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_parity16.json 2> $O/bench_parity16.err || { echo "parity16 failed"; tail -5 $O/bench_parity16.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_parity16.json'));print('parity16',d['value'],d['unet_ms_per_eval'],d['config']['options'])"
timeout -k 10 400 python bench.py --noise parity --batch 64 --steps 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_parity64.json 2> $O/bench_parity64.err || { echo "parity64 failed"; tail -5 $O/bench_parity64.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_parity64.json'));print('parity64',d['value'],d['unet_ms_per_eval'])"
timeout -k 10 400 python bench.py --batch 64 --steps 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/bench_device64.json 2> $O/bench_device64.err || { echo "device64 failed"; tail -5 $O/bench_device64.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_device64.json'));print('device64',d['value'],d['unet_ms_per_eval'])"
exit $rc
