#!/bin/bash
# Quick GPU check: selected GPU tests, the ES bench line without the side legs, and a kernel-trace
# profile of the eager pipeline. Each GPU step has its own limit; a failure ends the script.
#   tools/gpu_quick.sh "<pytest selection>" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
SEL=${1:-tests}
shift
if [ "$SEL" != none ]; then
    timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
        > $OUT/quick_tests.log 2>&1
    rc=$?
    tail -n 15 $OUT/quick_tests.log
    if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
fi
timeout -k 10 300 python bench.py --no-cpu --no-pmc --bpf-frames 0 --no-roofline "$@" > $OUT/quick_bench.json 2> $OUT/quick_bench.err
rc=$?
cat $OUT/quick_bench.json; tail -n 3 $OUT/quick_bench.err
if [ $rc -ne 0 ]; then echo "BENCH FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/qprof -o run --output-format csv -- \
    python3 bench.py --steps 1000 --no-graph --only-headline > $OUT/qprof.json 2> $OUT/qprof.log
rc=$?
if [ $rc -ne 0 ]; then echo "PROF FAILED rc=$rc"; tail -n 20 $OUT/qprof.log; exit $rc; fi
python3 tools/kstats.py $(find $OUT/qprof -name "*kernel_stats.csv" | head -1) 14
find $OUT/qprof -name "*_kernel_trace.csv" -delete
