"""Per-step kernel timeline (start offsets, durations, gaps) from a tools/gpu_timeline.sh trace."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), k))
rows.sort()
# steps start at zero2/setup after the raster+grad pair; print the last few steps
starts = [i for i, r in enumerate(rows) if r[2].startswith('setup_kernel')]
for si in starts[-4:-1]:
    t0 = rows[si][0]
    nxt = [i for i in starts if i > si]
    end = nxt[0] if nxt else len(rows)
    prev_end = None
    print("---- step at", si)
    for s, e, k in rows[si - 2:end]:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print("  %-28s start %+8.2f us  dur %7.2f us  gap %6.2f" % (k[:28], (s - t0) / 1e3, (e - s) / 1e3, gap))
        prev_end = e
