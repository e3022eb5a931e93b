#!/bin/bash
# Development A/B of the classifier search: k_cls_search's average duration (rocprofv3 kernel trace of
# tools/cls_probe.py) for the in-tree library and each named variant under pfilter-noetic_amd/var/.
#   tools/cls_ab.sh [variant ...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/cls_ab
mkdir -p $OUT
for v in tree "$@"; do
    lib=""
    [ "$v" != tree ] && lib=pfilter-noetic_amd/var/$v/libpfilter_hip.so
    PFILTER_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- \
        python3 tools/cls_probe.py --iters 50 > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.log; exit 1; }
    echo "== $v: $(grep ms/frame $OUT/$v.log)"
    python3 tools/kstats.py $(find $OUT/$v -name "*kernel_stats.csv" | head -1) 5
    find $OUT/$v -name "*_kernel_trace.csv" -delete
done
