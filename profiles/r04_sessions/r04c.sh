#!/bin/bash
# round 4: chunk-interval traces of the 8- and 16-chunk 256^2 layers (IFD_TRACE build), bench rehearsals at N = 2
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for L in "r256 128+0->128 skip0" "r256 128+128->128 skip0"; do
  IFD_LIB_PATH=$R/tools/abl/libifd_trace.so timeout -k 10 150 python tools/x3_trace.py "$L" > "$OUT/tr_$(echo $L | tr ' +>' '___').txt" 2>&1 || { echo "trace $L failed"; exit 1; }
done
echo traces ok
timeout -k 10 400 python bench.py --gpus 2 --steps 1 --warmup 1 --cpu-baseline-seconds 10 --no-profile > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err; echo "gpus2 rc=$?"
timeout -k 10 400 python bench.py --workload c4 --gpus 2 --global-batch 17 --steps 1 --warmup 0 --cpu-baseline-seconds 5 --no-profile > $OUT/bench_c4r.json 2> $OUT/bench_c4r.err; echo "c4 rehearsal rc=$?"
tail -c 700 $OUT/bench_gpus2.json; echo; tail -c 900 $OUT/bench_c4r.json
