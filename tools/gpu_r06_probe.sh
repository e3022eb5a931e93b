#!/bin/bash
# round 6: pop-engine variants (tools/mb/heap_pop) and per-level phase times of the partition tiers
# (variant build -DPF_TIE_PROF in pfilter-noetic_amd/var/tieprof6, tools/tie_prof.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06p}
mkdir -p $OUT
timeout -k 10 120 ./tools/mb/heap_pop 3 > $OUT/heap_pop.txt 2>&1 || { tail -5 $OUT/heap_pop.txt; exit 1; }
grep -v "^full" $OUT/heap_pop.txt | grep -v small
for a in "26000 -3500" "26000 -300" "12000 -2700"; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/tieprof6/libpfilter_hip.so timeout -k 10 120 python3 tools/tie_prof.py $a > "$OUT/tieprof_${a// /_}.txt" 2>&1 || { tail -5 "$OUT/tieprof_${a// /_}.txt"; exit 1; }
  echo "== $a"; cat "$OUT/tieprof_${a// /_}.txt"
done
