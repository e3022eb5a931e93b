"""Splits a rocprofv3 kernel trace of tools/tie_time.py into its tie sorts (each opens with
k_tie_compact) and prints, per case (3 calls each, in order), the median duration of every kernel.
    python3 tools/tie_trace.py <kernel_trace.csv> <case names...>"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
calls = []
for r in rows:
    m = re.search(r"k_tie_\w+", r["Kernel_Name"])
    if not m:
        continue
    short = m.group(0)
    # a sort opens with k_tie_compact (big path) or with k_tie_medium not preceded by k_tie_setup
    if short == "k_tie_compact" or (short == "k_tie_medium" and (not calls or calls[-1][-1][0] != "k_tie_split")
                                    and (not calls or calls[-1][-1][0] != "k_tie_setup")):
        calls.append([])
    if calls:
        calls[-1].append((short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0))
names = sys.argv[2:]
for i, nm in enumerate(names):
    group = calls[3 * i:3 * i + 3]
    if not group:
        break
    per = defaultdict(list)
    for c in group:
        acc = defaultdict(float)
        for k, us in c:
            acc[k] += us
        for k, us in acc.items():
            per[k].append(us)
    tot = sorted(sum(v for _, v in c) for c in group)[len(group) // 2]
    print("%-12s total %8.1f us  " % (nm, tot) + "  ".join("%s %.1f" % (k.replace("k_tie_", ""), sorted(v)[len(v) // 2])
                                                        for k, v in per.items()))
