#!/bin/bash
# round 6: the heap tier beside k_tie_local (PF_TIE_AUX=1) with fewer local workgroups (free CUs for the
# heap workgroups), full headline, alternated
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/auxab
mkdir -p $OUT
: > $OUT/summary.txt
run() {  # name lib aux
  local name=$1 lib=$2 aux=$3
  if [ -n "$lib" ]; then export PFILTER_HIP_LIB=$lib; else unset PFILTER_HIP_LIB; fi
  PF_TIE_AUX=$aux timeout -k 10 300 python3 -u bench.py --only-headline --steps 4521 --warmup 20 > $OUT/h_$name.json 2> $OUT/h_$name.err || { tail -5 $OUT/h_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/h_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d.get('stage_us'))" | tee -a $OUT/summary.txt
}
for r in 1 2; do
  run base_$r "" 0 && run aux_$r "" 1 && run lg192aux_$r pfilter-noetic_amd/var/lg192/libpfilter_hip.so 1 && run lg128aux_$r pfilter-noetic_amd/var/lg128/libpfilter_hip.so 1 && run lg192_$r pfilter-noetic_amd/var/lg192/libpfilter_hip.so 0 || exit 1
done
