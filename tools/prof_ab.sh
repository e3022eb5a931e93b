#!/bin/bash
# Per-kernel average durations of two libraries (eager launches), side by side.
#   tools/prof_ab.sh <variant>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pa_main -o run --output-format csv -- \
    python3 bench.py --steps 600 --no-cpu --no-graph --no-roofline --bpf-frames 0 > /dev/null 2>&1 || exit 1
PFILTER_HIP_LIB=pfilter-noetic_amd/var/$1/libpfilter_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/pa_var -o run --output-format csv -- \
    python3 bench.py --steps 600 --no-cpu --no-graph --no-roofline --bpf-frames 0 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
def load(d):
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("pf::(anonymous namespace)::", "").split("(")[0].split(" ")[-1]
        out[n] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3)
    return out
a, b = load("gpurun_out/pa_main"), load("gpurun_out/pa_var")
for k in sorted(set(a) | set(b), key=lambda k: -(a.get(k, (0, 0, 0))[2])):
    x, y = a.get(k, (0, 0, 0)), b.get(k, (0, 0, 0))
    print("%-32s main %5d x %7.2f us   var %5d x %7.2f us" % (k[:32], x[0], x[1], y[0], y[1]))
PY
