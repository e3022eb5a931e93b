"""Development: per-queue kernel totals from a rocprofv3 kernel trace (stage A and stage B of the pipeline
run on different streams, so on different queues).   python3 tools/stage_split.py run_kernel_trace.csv [frames]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
with open(path) as f:
    r = csv.DictReader(f)
    qkey = "Queue_Id" if "Queue_Id" in r.fieldnames else ("Stream_Id" if "Stream_Id" in r.fieldnames else None)
    for row in r:
        q = row.get(qkey, "?") if qkey else "?"
        name = row["Kernel_Name"].replace("pf::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        name = name.replace("void ", "").split("(")[0]
        d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
        tot[q][name] += d
        cnt[q][name] += 1
for q in sorted(tot, key=lambda k: -sum(tot[k].values())):
    s = sum(tot[q].values())
    print("queue %s: %.1f us per frame over %d frames" % (q, s / frames, frames))
    for name, v in sorted(tot[q].items(), key=lambda kv: -kv[1])[:14]:
        print("   %-40s %9.1f us/frame  calls %6d" % (name[:40], v / frames, cnt[q][name]))
