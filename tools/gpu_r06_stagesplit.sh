#!/bin/bash
# round 5-6: per-stage kernel time of the tie-order headline (eager launches, per-queue totals)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06ss}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/r06ss -o run --output-format csv -- \
    python3 bench.py --only-headline --no-cpu --no-graph --steps ${STEPS:-4521} > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 tools/stage_split.py $(ls /tmp/r06ss/*/run_kernel_trace.csv /tmp/r06ss/run_kernel_trace.csv 2>/dev/null | head -1) ${STEPS:-4521} > $OUT/split.txt
cat $OUT/split.txt
