#!/bin/bash
# Round-3 closing session: front-end parity tests, search A/B, the default bench line and its
# kernel-trace profile. A failed step ends the script.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
timeout -k 10 400 python -u -m pytest tests/test_gpu_cls.py tests/test_gpu_bpf.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/cls_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cls_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/cls_ab.sh "$@" || exit 1
PFILTER_HIP_LIB=pfilter-noetic_amd/var/clsstats/libpfilter_hip.so timeout -k 10 120 python3 tools/cls_probe.py --iters 3 \
    > gpurun_out/r03f/cls_stats.log 2>&1 || exit 1
grep CLS_STATS gpurun_out/r03f/cls_stats.log | tail -2
bash tools/gpu_r03.sh bench prof cls
