#!/bin/bash
# round 5: kernel trace of the whole tie-order headline (eager launches: the tracer's graph-replay fault,
# profiles/r05_graph_ring/)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r05ks}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --only-headline --no-cpu --no-graph > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
rm -f $OUT/trace/run_kernel_trace.csv
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv 25 > $OUT/kstats.txt
head -25 $OUT/kstats.txt
