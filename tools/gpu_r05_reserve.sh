#!/bin/bash
# round 5: stage-A CU reservation sweep of the tie-order headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r05rs
mkdir -p $OUT
for r in ${RESERVES:-128 192 224 64}; do
  PF_BENCH_STAGE_A_RESERVE=$r timeout -k 10 300 python3 -u bench.py --only-headline --no-cpu > $OUT/h_$r.json 2> $OUT/h_$r.err || { tail -5 $OUT/h_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/h_$r.json')); print('reserve $r', d['value'], d.get('stage_us'))"
done
