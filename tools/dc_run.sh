#!/bin/bash
# DCVC GPU check: its tests, then rocprofv3 kernel stats of the front end with curvedfilter on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_dcvc.py tests/test_gpu_cls.py > gpurun_out/dc_t.log 2>&1 || { tail -30 gpurun_out/dc_t.log; exit 1; }
tail -3 gpurun_out/dc_t.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dcvc_prof2 -o run --output-format csv -- python3 tools/cls_probe.py --iters 50 --dcvc > gpurun_out/dcvc_prof2.log 2>&1 || exit 1
grep ms/frame gpurun_out/dcvc_prof2.log
find gpurun_out/dcvc_prof2 -name "*_kernel_trace.csv" -delete
