#!/bin/bash
# round 6: configs[4] leg with stage B eager (the only handle) and graph-captured (a second handle alive,
# PF_GRAPH_AUTO), and the kitti11 leg
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06c4g}
mkdir -p $OUT
for name in alone other; do
  timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench, pfilter_amd as pa
keep = None
if '$name' == 'other':
    keep = pa.Odom_ES_EstimationClass(device=0, max_points=1000, map_capacity=1 << 16)
    keep.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
print(json.dumps(bench.configs4_leg(0, 100, 16, order='tie')))" > $OUT/c4_$name.json 2> $OUT/c4_$name.err || { tail -5 $OUT/c4_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_$name.json').read().strip().splitlines()[-1]); print('c4 $name', d['value'], d.get('stage_us'))"
done
timeout -k 10 400 python3 -u bench.py --sequences kitti11 --concurrent 4 > $OUT/kitti11.json 2> $OUT/kitti11.err || { tail -5 $OUT/kitti11.err; exit 1; }
tail -c 300 $OUT/kitti11.json
