#!/bin/bash
# round 6: configs[3] (KITTI 00-10 frame counts, one GPU, tie order) against the number of concurrent
# sequences K and the hardware queues per process (each run bounded below the silence limit)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/k11conc
mkdir -p $OUT
: > $OUT/summary2.txt
for cfg in ${CFGS:-"3 4" "4 4" "3 4" "4 4" "4 8" "3 8"}; do
  set -- $cfg; K=$1; Q=$2
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 150 python3 -u bench.py --sequences kitti11 --concurrent $K --warmup 5 > $OUT/k${K}_q$Q.json 2> $OUT/k${K}_q$Q.err || { echo "K=$K queues=$Q failed rc=$?" | tee -a $OUT/summary2.txt; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/k${K}_q$Q.json').read().strip().splitlines()[-1]); print('K=$K queues=$Q', d['value'], d.get('unit'))" | tee -a $OUT/summary2.txt
done
