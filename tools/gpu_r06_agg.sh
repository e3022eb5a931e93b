#!/bin/bash
# round 6: the odometry grid count with run aggregation (default) against one atomic per point (var/noagg):
# odometry tests, configs[4] leg and the headline, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06agg}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -2 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
for name in agg noagg agg2 noagg2; do
  LIB=""; [ "${name:0:5}" = "noagg" ] && LIB=pfilter-noetic_amd/var/noagg/libpfilter_hip.so
  PFILTER_HIP_LIB=$LIB timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
c4 = bench.configs4_leg(0, 100, 16, use_graph=1, order='tie')
print(json.dumps({'c4': c4['value']}))" > $OUT/c4_$name.json 2> $OUT/c4_$name.err || { tail -5 $OUT/c4_$name.err; exit 1; }
  PFILTER_HIP_LIB=$LIB timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/h_$name.json 2> $OUT/h_$name.err || { tail -5 $OUT/h_$name.err; exit 1; }
  echo "$name c4 $(tail -1 $OUT/c4_$name.json) headline $(python3 -c "import json; d=json.loads(open('$OUT/h_$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('stage_us'))")"
done
