#!/bin/bash
# round 5 session c: one-chunk-unit store deferral + wgrad_x3 cleanup: GPU tests; same-box layer A/B (base = X3_DEFER=4
# in-tree, d0 = no deferral); SQ/GRBM counter pass per library (cycles, MFMA busy, effective clock of the dominant
# conv); rocprofv3 kernel-trace stats of a short bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05c; mkdir -p $O
cd $R
PYTEST_X= bash tools/gpu_tests.sh; rc=$?; cp gpurun_out/gpu_tests.txt $O/; echo "tests rc=$rc"
for rep in 1 2; do
  for v in base d0; do
    if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
    timeout -k 10 120 python tools/layer_prof.py 16 3xf16 > $O/lp_${v}_$rep.txt 2>&1 || { echo "lp $v failed"; exit 1; }
    echo "$v.$rep $(tail -1 $O/lp_${v}_$rep.txt) | $(grep 'r256 128+0->128 skip0 ' $O/lp_${v}_$rep.txt | head -1 | cut -c60-) | $(grep 'r256 16+0->128' $O/lp_${v}_$rep.txt | head -1 | cut -c60-)"
  done
done
unset IFD_LIB_PATH
cd /tmp && export TMPDIR=/tmp
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for v in base d0; do
  if [ $v = base ]; then unset IFD_LIB_PATH; else export IFD_LIB_PATH=$R/tools/abl/libifd_$v.so; fi
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "conv_x3" -d $O/pmc_$v -o pmc --output-format csv -- \
     python $R/tools/one_eval.py 16 4 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed rc=$?"; tail -3 $O/pmc_$v.log; exit 1; }
  echo "pmc $v ok"
done
unset IFD_LIB_PATH
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- \
   python $R/bench.py --steps 1 --warmup 1 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 > $O/prof.log 2>&1 || { echo "rocprof trace failed rc=$?"; exit 1; }
echo "trace ok"
exit $rc
