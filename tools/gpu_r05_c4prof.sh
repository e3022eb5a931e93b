#!/bin/bash
# round 5: configs[4] in the tie order: the tie-sort tests, then a kernel trace of the frame probe
# (eager launches: the profiler's graph-replay fault, profiles/r05_graph_ring/)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/r05c4p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_parity_synced.py -k "tie or s128" -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/c4_probe.py 25 tie graph > $OUT/c4_tie.txt 2>&1 || { tail -5 $OUT/c4_tie.txt; exit 1; }
tail -4 $OUT/c4_tie.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 tools/c4_probe.py 25 tie eager > $OUT/c4_trace.txt 2>&1 || { tail -5 $OUT/c4_trace.txt; exit 1; }
rm -f $OUT/trace/run_kernel_trace.csv
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv 30 > $OUT/kstats.txt
head -30 $OUT/kstats.txt
