#!/bin/bash
# A/B of whole-pipeline variants (tools/build_variant.sh): odometry parity tests + bench frames/s.
#   tools/bench_ab.sh [variant ...]   ("" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in "" "$@"; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; fi
  echo "== ${v:-main} tests: $(timeout -k 10 300 python -m pytest -x -q -p no:cacheprovider tests/test_gpu_odom.py tests/test_gpu_knn.py -m gpu 2>&1 | tail -1)" || exit 1
  echo "== ${v:-main} $(timeout -k 10 200 python bench.py --no-cpu --no-roofline | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')" || exit 1
done
