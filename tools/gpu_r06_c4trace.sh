#!/bin/bash
# round 6: configs[4] in the tie order: a kernel trace of the eager frame probe, the stats and the
# condensed dispatch sequence of its last frames
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06c4t}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06c4t -o run --output-format csv -- \
    python3 tools/c4_probe.py ${FRAMES:-12} tie eager > $OUT/c4_trace.txt 2>&1 || { tail -5 $OUT/c4_trace.txt; exit 1; }
tail -4 $OUT/c4_trace.txt
TR=$(ls /tmp/r06c4t/*/run_kernel_trace.csv /tmp/r06c4t/run_kernel_trace.csv 2>/dev/null | head -1)
ST=$(ls /tmp/r06c4t/*/run_kernel_stats.csv /tmp/r06c4t/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kstats.py $ST 40 > $OUT/kstats.txt
python3 tools/stage_split.py $TR ${FRAMES:-12} > $OUT/split.txt
python3 tools/trace_tail.py $TR 1500 > $OUT/seq.txt
head -40 $OUT/kstats.txt
