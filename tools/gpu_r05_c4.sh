#!/bin/bash
# round 5: configs[4] in the tie order (deep big levels, huge depth-limit segments by one radix sort):
# the tie-sort GPU tests, the synced configs[4] parity tests, the frame-by-frame probe
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r05c4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_parity_synced.py -k "tie or s128" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?; tail -25 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/c4_probe.py 40 tie graph > $OUT/c4_tie.txt 2>&1 || { tail -5 $OUT/c4_tie.txt; exit 1; }
tail -12 $OUT/c4_tie.txt
