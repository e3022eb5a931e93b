#!/bin/bash
# round 6: rocprofv3 kernel statistics of (1) the graded roofline kernel alone (tools/knn_probe.py, config 5,
# k_knn_thick) and (2) the driver's bench command (eager launches: the tracer's graph-ring fault, r05)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06prof}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06knn -o run --output-format csv -- python3 tools/knn_probe.py --iters 50 > $OUT/knn_probe.txt 2>&1 || { tail -5 $OUT/knn_probe.txt; exit 1; }
cp $(ls /tmp/r06knn/*/run_kernel_stats.csv /tmp/r06knn/run_kernel_stats.csv 2>/dev/null | head -1) $OUT/knn_kernel_stats.csv
python3 tools/kstats.py $OUT/knn_kernel_stats.csv 8 > $OUT/knn_kernel_stats.txt
grep -v "^E2\|^W2" $OUT/knn_probe.txt | tail -2
head -4 $OUT/knn_kernel_stats.txt
timeout -k 10 800 rocprofv3 --kernel-trace --stats -d /tmp/r06kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-graph > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
cp $(ls /tmp/r06kt/*/run_kernel_stats.csv /tmp/r06kt/run_kernel_stats.csv 2>/dev/null | head -1) $OUT/kernel_stats.csv
python3 tools/kstats.py $OUT/kernel_stats.csv 40 > $OUT/kernel_stats.txt
head -12 $OUT/kernel_stats.txt
