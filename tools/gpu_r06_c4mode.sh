#!/bin/bash
# round 6: configs[4] leg, graph replay against eager launches, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06c4m}
mkdir -p $OUT
for name in g1 e1 g2 e2; do
  G=False; [ "${name:0:1}" = "g" ] && G=True
  timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
print(json.dumps(bench.configs4_leg(0, 100, 16, use_graph=$G, order='tie')))" > $OUT/c4_$name.json 2> $OUT/c4_$name.err || { tail -5 $OUT/c4_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_$name.json').read().strip().splitlines()[-1]); print('c4 $name', d['value'], d.get('stage_us'))"
done
