#!/bin/bash
# round-4 evidence on the GPU box: PMC passes over the frame path (stable order, as round 3's), a
# kernel trace of the tie-order pipeline over the whole sequence, then the default bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
ORDER=stable tools/frame_pmc.sh > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
echo "pmc done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 tools/tie_probe.py 4521 S64 tie > $OUT/probe_full.txt 2>&1 || { tail -5 $OUT/probe_full.txt; exit 1; }
rm -f $OUT/trace/run_kernel_trace.csv
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv 40 > $OUT/kstats.txt
head -12 $OUT/kstats.txt
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
