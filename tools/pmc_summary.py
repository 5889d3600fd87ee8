"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).
    python tools/pmc_summary.py gpurun_out/pmc7 [kernel-substring ...]
FETCH_SIZE is in KiB and on gfx950 counts half of a wide streaming read's bytes
(MI355X_MICROARCH.md, HBM): hbm_read_bytes = 2 * FETCH_SIZE * 1024.
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores."""
import csv, collections, glob, os, sys, json
root = sys.argv[1]
keys = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, '*', 'run_counter_collection.csv')):
    per = collections.defaultdict(float)
    names = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = (row['Dispatch_Id'], row['Counter_Name'])
            per[k] += float(row['Counter_Value'])
            names[row['Dispatch_Id']] = (row['Kernel_Name'], row['Grid_Size'],
                                         (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e6)
    for (d, cn), v in per.items():
        kname, grid, ms = names[d]
        acc[(kname, grid)][cn].append(v)
        acc[(kname, grid)]['ms'].append(ms)
out = {}
for (kname, grid), cs in acc.items():
    short = kname.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
    short = f"{short} grid={grid}"
    if keys and not any(k in short for k in keys):
        continue
    out[short] = {cn: sum(v) / len(v) for cn, v in cs.items()}
    out[short]['dispatches'] = max(len(v) for v in cs.values())
print(json.dumps(out, indent=1))
