#!/bin/bash
# round 5 session o: the 2-rank rehearsal's stdout after the process-group notice fix (one JSON line), and the
# C1 configuration (B = 1, 10-step DDIM cosine, eta 0.9) on the GPU in both geometries: single-image latency
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o; mkdir -p $O
cd $R
B="--cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0"
timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 $B > $O/bench_gpus2_rehearsal.json 2> $O/bench_gpus2_rehearsal.err || { echo "rehearsal failed"; tail -5 $O/bench_gpus2_rehearsal.err; exit 1; }
echo "stdout lines: $(wc -l < $O/bench_gpus2_rehearsal.json)"
python -c "import json;d=json.load(open('$O/bench_gpus2_rehearsal.json'));print('gpus2', d['value'], d['n_gpus'], d['n_ranks'], d['config'].get('parallelism'))" || exit 1
for nz in device parity; do
  timeout -k 10 300 python bench.py --batch 1 --ddim-steps 10 --eta 0.9 --noise $nz --steps 5 --warmup 2 $B > $O/bench_c1_$nz.json 2> $O/bench_c1_$nz.err || { echo "c1 $nz failed"; tail -3 $O/bench_c1_$nz.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c1_$nz.json'));print('c1 $nz', d['value'], d['ms_per_step'], d['unet_ms_per_eval'])"
done
# training: the output blocks' concat gradient written per source by the GroupNorm backward (no channel copy out of
# the C-wide gradient): the training GPU tests, the training bench twice, one traced step
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_train_fuse.py tests/test_gpu_train_gn.py tests/test_gpu_train_attn.py tests/test_gpu_train_gstat.py tests/test_gpu_blocks.py tests/test_gpu_configs.py -k "train or gn or attn or gstat or block or c5 or split or addend" > $O/train_tests.txt 2>&1; rc=$?
tail -3 $O/train_tests.txt; echo "train tests rc=$rc"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload train --batch 32 --steps 3 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 \
      > $O/train_$rep.json 2> $O/train_$rep.err || { echo "train failed"; tail -5 $O/train_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/train_$rep.json'));print('train rep $rep', d['value'], d['ms_per_step'], d['loss'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_train -o trace --output-format csv -- \
   python $R/bench.py --workload train --batch 32 --steps 2 --warmup 1 --fp32-exact-steps 0 --f16-steps 0 > $O/prof_train.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo "trace ok"
