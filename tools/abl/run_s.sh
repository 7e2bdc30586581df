#!/bin/bash
# development: SiLU-variant builds (tools/abl/libifd_s*.so): layer timings + parity subset per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-1 2 3}; do
  export IFD_LIB_PATH=$R/tools/abl/libifd_s$v.so
  timeout -k 10 120 python $R/tools/layer_prof.py 16 3xf16 > $R/gpurun_out/abls$v.txt 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_x3w.py $R/tests/test_gpu_x3.py::test_x3_unet_full $R/tests/test_gpu_x3.py::test_x3_matches_fp32_bench_batch -q --timeout 150 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/t_s$v.txt 2>&1
  rc=$?; [ $rc -gt 1 ] && { echo "tests $v rc=$rc"; exit $rc; }
  echo "variant $v ok (tests rc=$rc)"
done
