#!/bin/bash
# A/B of library variants on the ES legs (S64 headline, theta0, campus32, dense, dense_theta0), two
# alternating passes: frames/s per leg.   tools/leg_ab.sh [variant ...]   ("" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
for v in "" "$@"; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; else unset PFILTER_HIP_LIB; fi
  echo "== ${v:-main} $(timeout -k 10 300 python bench.py --no-cpu --no-roofline --no-pmc --bpf-frames 0 --steps 1000 --leg-frames 500 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], *[(k, d[k]["value"]) for k in ("theta0", "campus32", "dense", "dense_theta0") if k in d])')" || exit 1
done
done
