"""Per-(kernel, grid size) summary of a rocprofv3 kernel trace: calls and the
mean duration -- tells a level's instance of a kernel from another's.
    python tools/kgrid.py DIR [filter]"""
import csv, glob, os, re, sys
from collections import defaultdict

f = glob.glob(os.path.join(sys.argv[1], '**', '*kernel_trace.csv'), recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
acc = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    name = re.sub(r'\(.*', '', r['Kernel_Name'].replace('(anonymous namespace)::', '')
                  .replace('void ', ''))
    if flt not in name:
        continue
    key = (name, int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0))
    acc[key][0] += 1
    acc[key][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for (name, g), (n, us) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print(f"{name[:70]:70s} grid {g:>8d} calls {n:>5d} avg_us {us / n:9.1f} total_ms {us / 1e3:8.2f}")
