"""Print the rocprofv3 --stats kernel table(s) under a directory:
kernel, calls, average and total microseconds.  python3 tools/gpu/kstats.py DIR"""
import csv
import glob
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"), recursive=True)):
    print(f"== {os.path.relpath(f, sys.argv[1])}")
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us "
              f"{float(r['TotalDurationNs']) / 1e3:10.1f} us")
