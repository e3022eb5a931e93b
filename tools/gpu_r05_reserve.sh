#!/bin/bash
# round 5: stage-A CU reservation sweep of the tie-order headline (PF_STAGE_B_CU_EXCL: stage B on the
# reserved CUs only)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r05rs
mkdir -p $OUT
for cfg in ${CFGS:-128 192 64 128x 192x}; do
  r=${cfg%x}; x=""; [ "$cfg" != "$r" ] && x=1
  env ${x:+PF_STAGE_B_CU_EXCL=1} PF_STAGE_A_CU_RESERVE=$r timeout -k 10 300 python3 -u bench.py --only-headline --no-cpu > $OUT/h_$cfg.json 2> $OUT/h_$cfg.err || { tail -5 $OUT/h_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/h_$cfg.json')); print('cfg $cfg', d['value'], d.get('stage_us'))"
done
