#!/bin/bash
# A/B of the BPF chain (raw scan -> front end -> Odom_BPF) across library variants (tools/build_variant.sh
# or an older build under var/), two alternating passes: ES and BPF frames/s, and with the DCVC filter.
#   tools/bpf_ab.sh [variant ...]   ("" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
for v in "" "$@"; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; else unset PFILTER_HIP_LIB; fi
  echo "== ${v:-main} $(timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-pmc --leg-frames 0 --steps 500 --bpf-frames 1000 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["bpf"]["value"], d.get("bpf_dcvc", {}).get("value"))')" || exit 1
done
done
