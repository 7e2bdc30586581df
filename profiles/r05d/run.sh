#!/bin/bash
# round 5 session d: the fixed one-chunk-unit deferral: GPU tests, smoke, outputs vs d0 / d4m (bit-equal expected),
# same-box layer A/B (base; d0 = no deferral; d4m = no deferral for one-chunk units), trace of the input conv.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt gpurun_out/parity.json $O/; echo "tests rc=$rc"
[ $rc = 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python tools/abl/cmp_lib.py base > $O/cmp.txt 2>&1 || { echo "cmp failed"; exit 1; }
for v in d0 d4m; do
  IFD_LIB_PATH=$R/tools/abl/libifd_$v.so timeout -k 10 120 python tools/abl/cmp_lib.py $v --against base >> $O/cmp.txt 2>&1 || { echo "cmp $v failed"; exit 1; }
done
grep max-abs $O/cmp.txt
for rep in 1 2; do
  for v in base d0 d4m; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp_${v}_$rep.txt) | $(grep 'r256 128+0->128 skip0 ' $O/lp_${v}_$rep.txt | head -1 | cut -c60-) | $(grep 'r256 16+0->128' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
unset IFD_LIB_PATH
IFD_LIB_PATH=$R/tools/abl/libifd_trd4.so timeout -k 10 120 python tools/x3_trace.py 'r256 16+0->128' > $O/trace_in.txt 2>&1 || { echo "trace failed"; exit 1; }
grep -v amdgpu.ids $O/trace_in.txt
exit $rc
