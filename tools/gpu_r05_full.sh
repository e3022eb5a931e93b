#!/bin/bash
# round 5: the GPU suite, smoke, then the default bench line (and the kitti11 leg in the tie order)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r05f}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 1; }
  tail -1 $OUT/smoke.txt
fi
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'stage_us', d.get('stage_us'), 'c4', (d.get('configs4') or {}).get('value'), 'cpu', d['cpu_baseline']['value'], 'speedup', d.get('speedup_vs_cpu'))"
if [ -n "$KITTI11" ]; then
  timeout -k 10 400 python3 -u bench.py --sequences kitti11 --concurrent 4 > $OUT/kitti11.json 2> $OUT/kitti11.err || { tail -5 $OUT/kitti11.err; exit 1; }
  tail -c 400 $OUT/kitti11.json
fi
