"""Summarise rocprofv3 --pmc CSVs: median counter value per kernel (+ duration from the trace)."""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(root + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for f in sorted(glob.glob(root + '/p*/run_kernel_trace.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        dur[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, d in agg.items():
    if 'fillBuffer' in k:
        continue
    print(k, " median dur %.2f us" % statistics.median(dur[k]) if dur[k] else "")
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {statistics.median(v):14.1f}")
