#!/bin/bash
# rgbds-merge check on the GPU: the A/B tests, the headline bench line, the bucket phase probe and
# one steady-state frame of an eager kernel trace. Each GPU step under its own limit; stops at the
# first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_rgm.py \
    > $OUT/rgm.log 2>&1 || { tail -30 $OUT/rgm.log; exit 1; }
tail -2 $OUT/rgm.log
timeout -k 10 300 python3 bench.py --only-headline > $OUT/rgm_bench.json 2> $OUT/rgm_bench.err || { tail -5 $OUT/rgm_bench.err; exit 1; }
cat $OUT/rgm_bench.json
timeout -k 10 200 python3 -u tools/rgm_probe.py > $OUT/rgm_probe.log 2>&1 || { tail -5 $OUT/rgm_probe.log; exit 1; }
head -9 $OUT/rgm_probe.log
timeout -k 10 200 python3 -u tools/probe_lm2.py > $OUT/lm_probe.log 2>&1 || { tail -5 $OUT/lm_probe.log; exit 1; }
cat $OUT/lm_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/rtrace -o run --output-format csv -- \
    python3 bench.py --steps 300 --no-graph --only-headline > $OUT/rtrace.log 2>&1 || { tail -5 $OUT/rtrace.log; exit 1; }
python3 tools/trace_frame.py $(find $OUT/rtrace -name "*kernel_trace.csv" | head -1) 200 > $OUT/rgm_frame.txt
cat $OUT/rgm_frame.txt
find $OUT/rtrace -name "*.csv" -delete
