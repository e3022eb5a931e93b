#!/bin/bash
# Round check on the GPU: the whole -m gpu suite, the configs[3] multi-handle bench line, an eager
# kernel trace of the headline (one steady frame's timeline + rocprofv3 --stats summary). Each GPU
# step under its own limit; stops at the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider -m gpu --timeout 300 --timeout-method thread tests \
    > $OUT/full_gpu.log 2>&1 || { tail -30 $OUT/full_gpu.log; exit 1; }
tail -2 $OUT/full_gpu.log
timeout -k 10 250 python3 bench.py --sequences kitti11 > $OUT/k11.json 2> $OUT/k11.err || { tail -5 $OUT/k11.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k11.json'));print('k11', d['value'], d['unit'])"
rm -rf $OUT/rtrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rtrace -o run --output-format csv -- \
    python3 bench.py --steps 1000 --no-cpu --no-graph --only-headline > $OUT/rtrace.log 2>&1 || { tail -5 $OUT/rtrace.log; exit 1; }
python3 tools/trace_frame.py $(find $OUT/rtrace -name "*kernel_trace.csv" | head -1) 500 > $OUT/frame.txt
cat $OUT/frame.txt
cp $(find $OUT/rtrace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
find $OUT/rtrace -name "*.csv" -delete
