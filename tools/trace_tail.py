"""Development: the dispatch sequence of a rocprofv3 kernel trace, condensed (queue, kernel, start, duration,
gap to the previous dispatch on that queue), for the last N dispatches of the run or of one queue:
python3 tools/trace_tail.py run_kernel_trace.csv [N] [queue] > seq.txt"""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
want = sys.argv[3] if len(sys.argv) > 3 else None
rows = []
with open(path) as f:
    r = csv.DictReader(f)
    qkey = "Queue_Id" if "Queue_Id" in r.fieldnames else "Stream_Id"
    for row in r:
        name = row["Kernel_Name"].replace("pf::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        name = name.replace("void ", "").replace("pf::", "").split("(")[0]
        rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row[qkey], name))
rows.sort()
if want:
    rows = [x for x in rows if x[2] == want]
rows = rows[-n:]
last = {}
t0 = rows[0][0] if rows else 0
for s, e, q, name in rows:
    gap = (s - last[q]) / 1e3 if q in last else 0.0
    last[q] = e
    print("%12.1f q%-3s %-40s %9.1f us  gap %7.1f" % ((s - t0) / 1e3, q, name[:40], (e - s) / 1e3, gap))
