#!/bin/bash
# round 6: association team of 16 lanes up to 16384 queries (variant wide16k) against the default (8192):
# configs[4] leg (frames/s and the association kNN's roofline) and the dense S64V leg, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06wide}
mkdir -p $OUT
for name in base wide base2 wide2; do
  LIB=""; [ "${name:0:4}" = "wide" ] && LIB=pfilter-noetic_amd/var/wide16k/libpfilter_hip.so
  PFILTER_HIP_LIB=$LIB timeout -k 10 300 python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
c4 = bench.configs4_leg(0, 100, 16, use_graph=1, order='tie')
print(json.dumps({'c4': c4['value'], 'assoc_frac': c4['roofline']['frac'], 'assoc_ms': c4['roofline']['avg_kernel_ms']}))" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  echo "$name $(tail -1 $OUT/$name.json)"
done
