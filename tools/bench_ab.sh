#!/bin/bash
# A/B of whole-pipeline variants (tools/build_variant.sh or an older build under var/): bench frames/s,
# each library run twice in alternation so box drift shows.
#   tools/bench_ab.sh [variant ...]   ("" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for rep in ${REPS:-1 2}; do
for v in "" "$@"; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; else unset PFILTER_HIP_LIB; fi
  echo "== ${v:-main} $(timeout -k 10 200 python bench.py --only-headline | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("stage_us"))')" || exit 1
done
done
