#!/bin/bash
# round 6: the aux-stream heap launch (TieAux): tie tests, odometry tests, headline A/B (PF_TIE_AUX)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
for a in 1 0 1 0; do
  PF_TIE_AUX=$a timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/headline_aux$a.json 2> $OUT/headline_aux$a.err || { tail -5 $OUT/headline_aux$a.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/headline_aux$a.json').read().strip().splitlines()[-1]); print('aux $a value', d['value'], d.get('stage_us'))"
done
