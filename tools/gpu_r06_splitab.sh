#!/bin/bash
# round 6: the split / median round trips -- tie tests, configs[4]'s and configs[1]'s synced tie parity,
# then the configs[4] leg and the full headline alternated between the HEAD build (var/base) and this tree
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/splitab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?; tail -2 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
PF_PARITY_OUT=$OUT/parity timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_synced.py -x -q --timeout 500 --timeout-method thread -p no:cacheprovider -k "s128_2m_point_map_tie or configs1_S64-S64" > $OUT/pytest_sync.txt 2>&1
rc=$?; tail -2 $OUT/pytest_sync.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in base cur; do
    if [ $lib = base ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/base/libpfilter_hip.so; else unset PFILTER_HIP_LIB; fi
    timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
print(json.dumps(bench.configs4_leg(0, 100, 16, order='tie')))" > $OUT/c4_${lib}_$r.json 2> $OUT/c4_${lib}_$r.err || { tail -5 $OUT/c4_${lib}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_${lib}_$r.json').read().strip().splitlines()[-1]); print('c4 $lib $r', d['value'])"
    timeout -k 10 300 python3 -u bench.py --only-headline --steps 4521 --warmup 20 > $OUT/headline_${lib}_$r.json 2> $OUT/headline_${lib}_$r.err || { tail -5 $OUT/headline_${lib}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/headline_${lib}_$r.json').read().strip().splitlines()[-1]); print('headline $lib $r', d['value'], d.get('stage_us'))"
  done
done
