"""Print the k_dc_* kernels of rocprofv3 stats CSVs (tools/dc_run.sh)."""
import csv
import re
import sys

for f in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
    t = 0.0
    print(f)
    for r in rows:
        if 'k_dc' in r['Name']:
            us = float(r['AverageNs']) / 1e3
            t += us
            print('  %-40s %5s %7.1f' % (re.search(r'k_dc_\w+', r['Name']).group(0), r['Calls'], us))
    print('  k_dc_* total %.1f us' % t)
