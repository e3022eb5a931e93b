#!/bin/bash
# round 5: the dependence table's small path: A/B tests, the free-running tie-order parity, configs[4] timing
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r05dep}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rgm.py -k dep -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_dep.txt 2>&1
rc=$?; tail -6 $OUT/pytest_dep.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/c4_probe.py 25 tie graph > $OUT/c4_tie.txt 2>&1 || { tail -5 $OUT/c4_tie.txt; exit 1; }
tail -4 $OUT/c4_tie.txt
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_free.py tests/test_gpu_tie.py tests/test_gpu_parity_synced.py -k "s64t or headline or tie or s128" -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest_tie.txt 2>&1
  rc=$?; tail -25 $OUT/pytest_tie.txt; [ $rc -eq 0 ] || exit $rc
fi
