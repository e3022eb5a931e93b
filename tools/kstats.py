"""Top kernels of a rocprofv3 --stats kernel_stats.csv: tools/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    n = r['Name'].replace('pf::(anonymous namespace)::', '').replace('pf::', '')
    print("%-48s calls=%6s avg=%9.1f us  total=%8.2f ms" % (n.split('(')[0][:48], r['Calls'],
                                                          float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6))
