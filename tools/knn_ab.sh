#!/bin/bash
# A/B of kNN variants built by tools/build_variant.sh: parity tests, then the config-5 probe per team
#   tools/knn_ab.sh "<teams>" [variant ...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TEAMS=$1; shift
for v in "" "$@"; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; fi
  echo "== ${v:-main} tests: $(timeout -k 10 300 python -m pytest -x -q -p no:cacheprovider tests/test_gpu_knn.py -m gpu 2>&1 | tail -1)" || exit 1
  for t in $TEAMS; do
    echo "== ${v:-main} team $t $(timeout -k 10 120 python tools/knn_probe.py --team $t --iters 30 | cut -c1-40)" || exit 1
  done
done
