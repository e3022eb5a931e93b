#!/bin/bash
# Synced per-frame parity against the reference-faithful oracle (tests/test_gpu_parity_synced.py),
# summaries into gpurun_out/parity/. One GPU step with its own limit.
#   tools/gpu_parity.sh [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT/parity
cd $R
export PF_PARITY_OUT=$OUT/parity
K=${1:-synced}
T=${2:-tests/test_gpu_parity_synced.py}
timeout -k 10 1100 python -u -m pytest $T -m gpu -k "$K" -v -s -p no:cacheprovider \
    --timeout 900 --timeout-method thread > $OUT/parity_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|frame [0-9]+,|Error" $OUT/parity_tests.log | tail -n 40
exit $rc
