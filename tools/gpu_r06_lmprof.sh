#!/bin/bash
# rocprofv3 kernel statistics of the whole headline sequence (the frame path alone, eager launches: the
# tracer's graph-ring fault, r05) with the final library: k_lm_solve's average launch duration beside the
# in-kernel probe's span
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/lmprof
mkdir -p $OUT
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/lmkt -o run --output-format csv -- python3 bench.py --only-headline --no-graph --steps 4521 --warmup 20 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cp $(ls /tmp/lmkt/*/run_kernel_stats.csv /tmp/lmkt/run_kernel_stats.csv 2>/dev/null | head -1) $OUT/kernel_stats.csv
python3 tools/kstats.py $OUT/kernel_stats.csv 30 > $OUT/kernel_stats.txt
head -14 $OUT/kernel_stats.txt
