#!/bin/bash
# round 5: the hand-scheduled LDS pop engine: tie-sort tests, tie parity (synced + free), windows probe
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r05h2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_rgm.py tests/test_gpu_parity_free.py tests/test_gpu_parity_synced.py -k "tie or dep or s64t or headline or s128 or every_frame" -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?; tail -30 $OUT/pytest.txt | grep -E "PASS|FAIL|Error|passed|failed"; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python3 -u bench.py --only-headline --no-cpu > $OUT/headline.json 2> $OUT/headline.err || { tail -5 $OUT/headline.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/headline.json')); print('value', d['value'], d.get('stage_us'))"
fi
