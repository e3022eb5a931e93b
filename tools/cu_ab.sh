#!/bin/bash
# Development: ES and BPF frame rates for stage-A CU reservations (PF_STAGE_A_CU_RESERVE), two passes.
#   tools/cu_ab.sh "0 32 64" 
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
for r in $1; do
  echo "== reserve $r $(PF_STAGE_A_CU_RESERVE=$r timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-pmc --leg-frames 0 --steps 2000 --bpf-frames 500 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["bpf"]["value"])')" || exit 1
done
done
