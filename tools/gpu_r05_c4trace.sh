#!/bin/bash
# round 5: configs[4] in the tie order: frame probe (graph) + kernel trace of the eager probe
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r05c4t}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/c4_probe.py 25 tie graph > $OUT/c4_tie.txt 2>&1 || { tail -5 $OUT/c4_tie.txt; exit 1; }
tail -4 $OUT/c4_tie.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 tools/c4_probe.py 25 tie eager > $OUT/c4_trace.txt 2>&1 || { tail -5 $OUT/c4_trace.txt; exit 1; }
rm -f $OUT/trace/run_kernel_trace.csv
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv 30 > $OUT/kstats.txt
head -30 $OUT/kstats.txt
