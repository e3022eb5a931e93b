#!/bin/bash
# round 6: the whole GPU suite (synced parity summaries written under $OUT/parity) and smoke
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06t}
mkdir -p $OUT
PF_PARITY_OUT=$OUT/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
