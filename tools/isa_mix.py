"""Instruction mix of the loops of a kernel in a hipcc -save-temps .s file.
    python tools/isa_mix.py FILE.s SYMBOL_SUBSTRING
For every backward branch (a loop) prints its length and the counts of fp64
VALU, other VALU, DPP movs, LDS, global/buffer, scalar and waitcnt
instructions -- the VALU issue budget of a march step at a glance.
"""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = None
for i, ln in enumerate(lines):
    if re.match(r"^_Z\S*:", ln) and sub in ln.split(":")[0]:
        start = i
        break
if start is None:
    sys.exit(f"no symbol containing {sub}")
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
print(lines[start].split(":")[0][:120])
labels = {}
for i, ln in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", ln)
    if m:
        labels[m.group(1)] = i


def classify(op):
    if op.startswith("v_") and "_f64" in op:
        return "valu_f64"
    if op.startswith("v_") and "dpp" in op:
        return "dpp"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu/smem"
    return None


def mix(a, b):
    c = collections.Counter()
    ops = collections.Counter()
    for ln in body[a:b]:
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        k = classify(op)
        if k:
            c[k] += 1
            if k.startswith("valu"):
                ops[op] += 1
    return c, ops


tot, totops = mix(0, len(body))
print("whole kernel:", dict(tot))
for i, ln in enumerate(body):
    m = re.match(r"\s*s_cbranch_\w+\s+(\.LBB\d+_\d+)", ln) or re.match(r"\s*s_branch\s+(\.LBB\d+_\d+)", ln)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        a = labels[m.group(1)]
        c, ops = mix(a, i + 1)
        if sum(c.values()) < 50:
            continue
        print(f"loop {m.group(1)} lines {a}-{i}: {dict(c)}")
        print("   top VALU:", ops.most_common(14))
