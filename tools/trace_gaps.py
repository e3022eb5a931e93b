"""Stage-B timeline statistics from a rocprofv3 kernel trace of a graph-mode bench run: per frame, the
span from the first stage-B kernel's start to the last one's end, the busy time (sum of kernel
durations), the idle time between consecutive stage-B kernels (launch gaps), and the idle time
between frames; medians over the steady frames.
  tools/trace_gaps.py run_kernel_trace.csv [first_frame] [frames]"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 200
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 500
heads = [i for i, r in enumerate(rows) if 'PredictTail' in r['Kernel_Name']]   # stage B's first kernel
qb = rows[heads[0]]['Queue_Id']
span, busy, gaps, between, per_kernel_gap = [], [], [], [], {}
for k in range(f0, min(f0 + nf, len(heads) - 1)):
    ks = [r for r in rows[heads[k]:heads[k + 1]] if r['Queue_Id'] == qb]
    s = [int(r['Start_Timestamp']) for r in ks]
    e = [int(r['End_Timestamp']) for r in ks]
    span.append((max(e) - s[0]) / 1000)
    busy.append(sum(b - a for a, b in zip(s, e)) / 1000)
    g = 0.0
    for i in range(1, len(ks)):
        d = max(0, s[i] - max(e[:i])) / 1000
        g += d
        nm = ks[i]['Kernel_Name'].replace('pf::(anonymous namespace)::', '').split('(')[0][:36]
        per_kernel_gap.setdefault(nm, []).append(d)
    gaps.append(g)
    nxt = int(rows[heads[k + 1]]['Start_Timestamp'])
    between.append((nxt - max(e)) / 1000)
med = st.median
print("stage-B frames %d (queue %s): span %.1f us, busy %.1f, gaps inside %.1f, idle before next frame %.1f, "
      "period %.1f" % (len(span), qb, med(span), med(busy), med(gaps), med(between), med(span) + med(between)))
for nm, v in sorted(per_kernel_gap.items(), key=lambda x: -med(x[1])):
    print("  gap before %-36s median %.2f us (n=%d)" % (nm, med(v), len(v)))
