#!/bin/bash
# Round-3 measurement session on one GPU box: the default bench line, a kernel-trace profile of the
# eager frame path, the BPF front end's kernel-trace profile, the BPF concurrency probe and the frame
# PMC passes. Every GPU step has its own limit; a crash / abort / timeout ends the script (no retries).
#   tools/gpu_r03.sh [bench] [prof] [cls] [stats] [conc] [pmc]   (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${R03_OUT:-r03}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
STEPS="$*"
[ -z "$STEPS" ] && STEPS="bench prof cls stats conc pmc"
want() { case " $STEPS " in *" $1 "*) return 0 ;; *) return 1 ;; esac; }

if want bench; then
    timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
    rc=$?
    cat $OUT/bench.json; tail -n 3 $OUT/bench.err
    [ $rc -ne 0 ] && { echo "BENCH FAILED rc=$rc"; exit $rc; }
fi
if want prof; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 1000 --no-graph --only-headline > $OUT/prof_bench.json 2> $OUT/prof.log
    rc=$?
    [ $rc -ne 0 ] && { echo "PROF FAILED rc=$rc"; tail -n 20 $OUT/prof.log; exit $rc; }
    python3 tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 20
fi
if want cls; then
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/cls_prof -o run --output-format csv -- \
        python3 tools/cls_probe.py --iters 50 > $OUT/cls_prof.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "CLS PROF FAILED rc=$rc"; tail -n 20 $OUT/cls_prof.log; exit $rc; }
    grep ms/frame $OUT/cls_prof.log
    python3 tools/kstats.py $(find $OUT/cls_prof -name "*kernel_stats.csv" | head -1) 8
    find $OUT/cls_prof -name "*_kernel_trace.csv" -delete
fi
if want stats; then   # the search's work counters (variant built with -DPF_DEV_CLS_STATS)
    PFILTER_HIP_LIB=pfilter-noetic_amd/var/clsstats/libpfilter_hip.so timeout -k 10 200 \
        python3 tools/cls_probe.py --iters 3 > $OUT/cls_stats.log 2>&1
    rc=$?
    grep CLS_STATS $OUT/cls_stats.log | tail -n 3
    [ $rc -ne 0 ] && { echo "STATS FAILED rc=$rc"; tail -n 20 $OUT/cls_stats.log; exit $rc; }
fi
if want conc; then
    timeout -k 10 300 python3 tools/bpf_conc_probe.py 300 > $OUT/bpf_conc.log 2>&1
    rc=$?
    cat $OUT/bpf_conc.log | tail -n 4
    [ $rc -ne 0 ] && { echo "CONC FAILED rc=$rc"; exit $rc; }
fi
if want pmc; then
    timeout -k 10 700 bash tools/frame_pmc.sh > $OUT/frame_pmc.log 2>&1
    rc=$?
    tail -n 30 $OUT/frame_pmc.log
    [ $rc -ne 0 ] && { echo "PMC FAILED rc=$rc"; exit $rc; }
fi
du -sh $OUT
