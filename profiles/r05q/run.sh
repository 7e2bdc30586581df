#!/bin/bash
# round 5 session q: single-image latency (C1, B = 1): HIP graph replay vs eager for one fused DDIM step, and a
# kernel trace of the C1 bench (kernel time vs wall: the launch gaps)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05q; mkdir -p $O
cd $R
timeout -k 10 300 python tools/graph_probe.py 50 1 > $O/graph_probe_b1.txt 2>&1 || { echo "probe failed"; tail -5 $O/graph_probe_b1.txt; exit 1; }
tail -3 $O/graph_probe_b1.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o trace --output-format csv -- \
   python $R/bench.py --batch 1 --ddim-steps 10 --eta 0.9 --steps 5 --warmup 2 --cpu-baseline-seconds 0 --fp32-exact-steps 0 --f16-steps 0 --no-profile > $O/prof_c1.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "trace ok"; tail -1 $O/prof_c1.log | cut -c1-300
