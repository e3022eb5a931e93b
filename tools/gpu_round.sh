#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench, rocprofv3 kernel-trace stats, kNN PMC passes.
# Every GPU step has its own time limit; a crash / abort / timeout ends the script (no retries).
#   tools/gpu_round.sh [tests|bench|all]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
WHAT=${1:-all}

fatal() {  # exit codes that mean the GPU step crashed or hung
    case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
    timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
    rc=$?
    tail -n 30 $OUT/pytest_gpu.log
    if fatal $rc || [ $rc -gt 1 ]; then echo "PYTEST CRASHED rc=$rc"; exit $rc; fi
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    rc=$?
    tail -n 5 $OUT/smoke.log
    if [ $rc -ne 0 ]; then echo "SMOKE FAILED rc=$rc"; exit $rc; fi
fi

if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
    rc=$?
    cat $OUT/bench.json; tail -n 5 $OUT/bench.err
    if [ $rc -ne 0 ]; then echo "BENCH FAILED rc=$rc"; exit $rc; fi
    # kernel durations: eager launches (--no-graph) so every kernel is traced individually
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 1000 --no-graph --only-headline > $OUT/prof_bench.json 2> $OUT/prof.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "PROF FAILED rc=$rc"; tail -n 20 $OUT/prof.log; exit $rc; fi
    echo prof ok
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
        python3 tools/knn_probe.py --iters 10 > $OUT/pmc_fetch.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "PMC FETCH FAILED rc=$rc"; tail -n 20 $OUT/pmc_fetch.log; exit $rc; fi
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
        python3 tools/knn_probe.py --iters 10 > $OUT/pmc_write.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "PMC WRITE FAILED rc=$rc"; tail -n 20 $OUT/pmc_write.log; exit $rc; fi
    echo pmc ok
    # the BPF front end (ground_seg + featureExtract) alone: per-kernel durations
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/cls_prof -o run --output-format csv -- \
        python3 tools/cls_probe.py --iters 50 > $OUT/cls_prof.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "CLS PROF FAILED rc=$rc"; tail -n 20 $OUT/cls_prof.log; exit $rc; fi
    grep ms/frame $OUT/cls_prof.log
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/dcvc_prof -o run --output-format csv -- \
        python3 tools/cls_probe.py --iters 50 --dcvc > $OUT/dcvc_prof.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "DCVC PROF FAILED rc=$rc"; tail -n 20 $OUT/dcvc_prof.log; exit $rc; fi
    grep ms/frame $OUT/dcvc_prof.log
    # the global map (LaserMappingClass) updates
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/map_prof -o run --output-format csv -- \
        python3 tools/map_probe.py --frames 200 > $OUT/map_prof.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "MAP PROF FAILED rc=$rc"; tail -n 20 $OUT/map_prof.log; exit $rc; fi
    grep "per update" $OUT/map_prof.log
    # gpurun copies back at most 64 MiB: keep the stats summaries, drop the per-dispatch traces
    find $OUT -name "*_kernel_trace.csv" -size +2M -not -path "$OUT/prof/*" -delete
    du -sh $OUT
fi
