#!/bin/bash
# round 5: per-level phase times of the partition tiers on rgbds-like inputs (prof build)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r05tp
mkdir -p $OUT
for v in tieprof_old tieprof_new; do for a in "26000 -3500" "26000 -300" "12000 -2700" "60000 13"; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so timeout -k 10 120 python3 tools/tie_prof.py $a > "$OUT/${v}_${a// /_}.txt" 2>&1 || { cat "$OUT/${v}_${a// /_}.txt" | tail -5; exit 1; }
  echo "== $v $a"; cat "$OUT/${v}_${a// /_}.txt"
done; done
