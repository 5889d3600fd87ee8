"""Print a rocprofv3 --kernel-trace --stats summary (kernel_stats.csv) compactly.
    python tools/ktrace_summary.py DIR [top]"""
import csv, glob, os, sys
f = glob.glob(os.path.join(sys.argv[1], '**', '*kernel_stats.csv'), recursive=True)[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for r in list(csv.DictReader(open(f)))[:top]:
    name = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
    print(f"{name[:48]:48s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f} "
          f"total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
