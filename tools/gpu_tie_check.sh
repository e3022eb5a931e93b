#!/bin/bash
# tie-order sort: GPU tests, then the ES pipeline probe (tie off / on) and a kernel-trace profile of
# the tie mode. Each GPU step has its own limit; a failure ends the script.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/tie; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tie.py ${TIE_TESTS:-} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -n 12 $OUT/tests.log; [ $rc -ne 0 ] && { echo "TESTS FAILED rc=$rc"; exit $rc; }
timeout -k 10 300 python -u tools/tie_probe.py ${TIE_N:-1000} > $OUT/probe.txt 2>&1
rc=$?; cat $OUT/probe.txt; [ $rc -ne 0 ] && { echo "PROBE FAILED rc=$rc"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/tie_probe.py 300 S64 tie > $OUT/prof.txt 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "PROF FAILED rc=$rc"; tail -5 $OUT/prof.txt; exit $rc; }
python3 tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 30 > $OUT/kstats.txt; cat $OUT/kstats.txt
find $OUT/prof -name "*_kernel_trace.csv" -delete
