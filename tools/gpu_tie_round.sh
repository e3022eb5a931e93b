#!/bin/bash
# tie-order round check: GPU tests of the touched areas, the sort alone on synthetic key sets, its
# per-phase profile, the ES pipeline in both orders and a kernel-trace profile of the tie mode.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/tier; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_fe.py tests/test_gpu_shim.py tests/test_gpu_host_io.py ${EXTRA_TESTS:-} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -n 5 $OUT/tests.log; [ $rc -ne 0 ] && { echo "TESTS FAILED rc=$rc"; exit $rc; }
TIE_LEVELS="0" tools/gpu_tie_time.sh > $OUT/tie_time.txt 2>&1 || { cat $OUT/tie_time.txt; exit 1; }
cat $OUT/tie_time.txt
for a in "2000 13" "45000 13" "25700 -3700"; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/tieprof/libpfilter_hip.so timeout -k 10 120 python3 tools/tie_prof.py $a > $OUT/prof_${a// /_}.txt 2>&1 || { echo "PROF FAILED"; exit 1; }
  head -14 $OUT/prof_${a// /_}.txt
done
timeout -k 10 300 python -u tools/tie_probe.py ${TIE_N:-1000} > $OUT/probe.txt 2>&1
rc=$?; cat $OUT/probe.txt; [ $rc -ne 0 ] && { echo "PROBE FAILED rc=$rc"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/tie_probe.py 300 S64 tie > $OUT/rocprof.txt 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "ROCPROF FAILED rc=$rc"; tail -5 $OUT/rocprof.txt; exit $rc; }
python3 tools/kstats.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 32 > $OUT/kstats.txt; cat $OUT/kstats.txt
find $OUT/prof -name "*_kernel_trace.csv" -delete
