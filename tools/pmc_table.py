"""Average each PMC counter per dispatch of the kernels whose name contains a filter string.
  python3 tools/pmc_table.py <dir with rocprofv3 csv passes> <kernel substring>"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root, filt = sys.argv[1], sys.argv[2]
    acc = defaultdict(list)
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if filt in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(acc):
        v = acc[k]
        print("%-28s n=%-4d mean=%.6g" % (k, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main()
