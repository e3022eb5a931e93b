#!/bin/bash
# round 6: tie tests, configs[4]'s synced tie parity, the configs[4] leg and the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06c4ab}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
PF_TIE_HS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_tie.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_hs0.txt 2>&1
rc=$?; tail -2 $OUT/pytest_hs0.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "$PARITY" ]; then
  date +%s > $OUT/t0
  PF_PARITY_OUT=$OUT/parity timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_synced.py -x -q -s --timeout 800 --timeout-method thread -p no:cacheprovider -k "s128_2m_point_map_tie" > $OUT/pytest_c4.txt 2>&1
  rc=$?; date +%s >> $OUT/t0; tail -3 $OUT/pytest_c4.txt; [ $rc -eq 0 ] || exit $rc
fi
for name in ${RUNS:-a}; do
  timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
print(json.dumps(bench.configs4_leg(0, 100, 16, order='tie')))" > $OUT/c4_$name.json 2> $OUT/c4_$name.err || { tail -5 $OUT/c4_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_$name.json').read().strip().splitlines()[-1]); print('c4 $name', d['value'], d.get('stage_us'))"
  timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/headline_$name.json 2> $OUT/headline_$name.err || { tail -5 $OUT/headline_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/headline_$name.json').read().strip().splitlines()[-1]); print('headline $name', d['value'], d.get('stage_us'))"
done
