#!/bin/bash
# round-4 evidence on the GPU box: PMC passes over the frame path (stable order, as round 3's), a
# kernel trace of the tie-order pipeline over the whole sequence, then the default bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
[ -n "$SKIP_PMC" ] || ORDER=stable tools/frame_pmc.sh > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
echo "pmc done"
# eager launches: rocprofv3's kernel trace of this image faults on the host side in hipGraphLaunch
# after a few hundred replays of these graphs. Round 5 reproduced it without the pipeline
# (tools/mb/graph_ring.hip, profiles/r05_graph_ring/): the tool's queue-intercept callback reads a graph's
# packet batch linearly past the end of the 16384-packet AQL ring when the batch straddles the wrap
# (15 kernels per graph fault at the first wrap, 16 never do)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --only-headline --no-graph --steps ${TRACE_N:-2000} --warmup 20 > $OUT/trace_bench.json 2> $OUT/trace_bench.err \
    || { tail -5 $OUT/trace_bench.err; exit 1; }
rm -f $OUT/trace/run_kernel_trace.csv
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv 40 > $OUT/kstats.txt
head -12 $OUT/kstats.txt
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
