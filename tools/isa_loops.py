"""Per-loop census of one kernel in an hipcc -S listing: instructions, VALU,
scratch (spill) accesses, LDS ops, barriers.
    python tools/isa_loops.py k.s MANGLED_NAME_SUBSTRING"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
starts = [m.start() for m in re.finditer(r"^(_Z\S+):", s, re.M)]
for st in starts:
    name = s[st:s.index(":", st)]
    if key not in name:
        continue
    body = s[st:s.index(".Lfunc_end", st)].split("\n")
    # innermost loop regions: label lines with 'Loop Header: Depth=N' start a loop
    heads = [(k, l) for k, l in enumerate(body) if "Loop Header" in l or "=>This Inner Loop" in l]
    print(name[:120])
    marks = [k for k, l in enumerate(body) if l.startswith(".LBB") and "Depth=2" in l]
    # group consecutive Depth=2 lines by their header
    groups = collections.OrderedDict()
    for k in marks:
        m = re.search(r"Header=(BB\d+_\d+)", body[k])
        h = m.group(1) if m else body[k].split(":")[0].lstrip(".L")
        groups.setdefault(h, []).append(k)
    for h, ks in groups.items():
        a, b = min(ks), max(ks) + 1
        while b < len(body) and not body[b].startswith(".LBB"):
            b += 1
        c = collections.Counter()
        for l in body[a:b]:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            c[t[0]] += 1
        valu = sum(v for k2, v in c.items() if k2.startswith("v_"))
        scr = sum(v for k2, v in c.items() if k2.startswith("scratch_"))
        ds = sum(v for k2, v in c.items() if k2.startswith("ds_"))
        f64 = sum(v for k2, v in c.items() if k2.endswith("_f64"))
        print(f"  loop {h}: lines {a}-{b} VALU {valu} f64 {f64} scratch {scr} ds {ds} "
              f"barrier {c['s_barrier']} vmcnt0 {sum('vmcnt(0)' in l for l in body[a:b])}")
