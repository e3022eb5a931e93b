#!/bin/bash
# round 6: the driver's bench command (--steps 20 --warmup 5: headline + every leg + full_sequence), the
# kitti11 leg, and a rocprofv3 kernel-trace --stats pass over the same bench command (PMC passes off: the
# bench's own traffic pass runs rocprofv3 itself)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06b}
mkdir -p $OUT
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); fs=d.get('full_sequence') or {}
print('value', d['value'], 'speedup', d.get('speedup_vs_cpu'), 'full', fs.get('value'), fs.get('speedup_vs_cpu'), (fs.get('cpu_baseline') or {}).get('value'), fs.get('stage_us'))
print('c4', (d.get('configs4') or {}).get('value'), 'bpf', (d.get('bpf') or {}).get('value'), 'wt2', (d.get('weight2') or {}).get('value'), 'roof', d['roofline']['frac'])"
if [ -n "$KITTI11" ]; then
  timeout -k 10 400 python3 -u bench.py --sequences kitti11 --concurrent 4 > $OUT/kitti11.json 2> $OUT/kitti11.err || { tail -5 $OUT/kitti11.err; exit 1; }
  tail -c 300 $OUT/kitti11.json
fi
if [ -n "$PROF" ]; then
  timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/r06kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-graph > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
  cp $(ls /tmp/r06kt/*/run_kernel_stats.csv /tmp/r06kt/run_kernel_stats.csv 2>/dev/null | head -1) $OUT/kernel_stats.csv
  python3 tools/kstats.py $OUT/kernel_stats.csv > $OUT/kernel_stats.txt 2>/dev/null || head -30 $OUT/kernel_stats.csv > $OUT/kernel_stats.txt
  head -25 $OUT/kernel_stats.txt
fi
