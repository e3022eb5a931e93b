#!/bin/bash
# round 5: the pop engine A/B (PF_HEAP_ENGINE 1 / 2, prof builds) on one depth-0 segment, then the GPU suite
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r05h
mkdir -p $OUT
for v in ${VARIANTS:-heap1 heap2}; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so timeout -k 10 120 python3 tools/heap_prof.py ${SIZES:-3000 15000} > $OUT/$v.txt 2>&1 || { tail -5 $OUT/$v.txt; exit 1; }
  echo "== $v"; cat $OUT/$v.txt
done
[ -n "$SKIP_TESTS" ] && exit 0
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider --durations=15 > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -25 $OUT/pytest_gpu.txt; exit $rc
