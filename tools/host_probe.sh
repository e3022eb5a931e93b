#!/bin/bash
# Frame rate and the host's enqueue time per frame, graph replay and eager launches.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  timeout -k 10 200 python bench.py --no-cpu --no-roofline --bpf-frames 0 --leg-frames 0 "$@" > gpurun_out/hp.json 2> gpurun_out/hp.err || { tail -5 gpurun_out/hp.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hp.json')); print(d['value'], d['config']['host_enqueue_us_per_frame'], d['stage_us'])"
}
echo "graph:"; run
echo "eager:"; run --no-graph
