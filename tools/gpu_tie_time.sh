#!/bin/bash
# tie-order sort alone on synthetic key sets, per-kernel durations per call (tools/tie_time.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/tiet; rm -rf $OUT; mkdir -p $OUT
CASES="vg11k_rand vg14k_rand vg45k_rand vg45k_runs4 distinct11k rg22k+3.7k rg10k+3.3k"
for lv in ${TIE_LEVELS:-2}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/prof$lv -o run --output-format csv -- python3 tools/tie_time.py $lv > $OUT/run$lv.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "RUN FAILED rc=$rc"; tail -20 $OUT/run$lv.txt; exit $rc; }
  echo "levels $lv"; python3 tools/tie_trace.py $(find $OUT/prof$lv -name "*kernel_trace.csv" | head -1) $CASES | tee $OUT/times$lv.txt
  find $OUT/prof$lv -name "*_kernel_trace.csv" -delete
done
