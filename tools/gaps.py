"""Launch gaps from a rocprofv3 kernel trace: for the last K V-cycles of the
trace (a cycle ends with the cross pass's edge kernel), each kernel's
duration and the idle time before it (previous kernel's end -> its start).
    python tools/gaps.py run_kernel_trace.csv [--cycles 3]"""
import argparse, csv, re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument('trace')
ap.add_argument('--cycles', type=int, default=3)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))


def short(name):
    name = re.sub(r'\(.*', '', name)
    return name[:60]


ends = [i for i, r in enumerate(rows) if 'k_xsmooth' in r['Kernel_Name']]
# the cross pass is two launches (interior, edges): a cycle ends at the second
ends = [i for i in ends if i + 1 >= len(rows) or 'k_xsmooth' not in rows[i + 1]['Kernel_Name']]
if len(ends) < a.cycles + 1:
    raise SystemExit(f'only {len(ends)} cycles in the trace')
lo, hi = ends[-a.cycles - 1] + 1, ends[-1] + 1
tot_busy = tot_gap = 0.0
per = defaultdict(lambda: [0, 0.0, 0.0])
for i in range(lo, hi):
    r, p = rows[i], rows[i - 1]
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - int(p['End_Timestamp'])) / 1e3
    dur = (e - s) / 1e3
    tot_busy += dur
    tot_gap += gap
    if i < lo + (hi - lo) // a.cycles:
        print(f"{dur:9.1f} us  gap {gap:7.1f} us  {short(r['Kernel_Name'])}  grid {r.get('Grid_Size', '')}")
span = (int(rows[hi - 1]['End_Timestamp']) - int(rows[lo - 1]['End_Timestamp'])) / 1e3
print(f"per cycle: span {span / a.cycles:.1f} us, busy {tot_busy / a.cycles:.1f} us, "
      f"gaps {tot_gap / a.cycles:.1f} us, launches {(hi - lo) / a.cycles:.0f}")
