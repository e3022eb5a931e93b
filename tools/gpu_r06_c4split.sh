#!/bin/bash
# round 6: configs[4] as bench.py's leg runs it (pipelined, eager launches so the trace sees every kernel):
# per-queue kernel totals and the dispatch sequence of its last frames
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06c4s}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r06c4s -o run --output-format csv -- \
    python3 -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
print(json.dumps(bench.configs4_leg(0, ${FRAMES:-40}, 16, use_graph=${GRAPH:-False}, order='tie')))" > $OUT/c4.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
TR=$(ls /tmp/r06c4s/*/run_kernel_trace.csv /tmp/r06c4s/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/stage_split.py $TR $((${FRAMES:-40} + 24)) > $OUT/split.txt
python3 tools/trace_tail.py $TR 1500 > $OUT/seq.txt
head -30 $OUT/split.txt
python3 -c "import json; d=json.loads(open('$OUT/c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d.get('stage_us'))"
