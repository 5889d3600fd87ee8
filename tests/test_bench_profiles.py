"""CPU: bench.py's PMC-traffic lookup stays wired to the kernels it names.

bench.KERNEL_IDS spells the dominant pass's template instances as rocprofv3
prints them; a template parameter added to k_xsmooth changes those names and
would silently turn the bench line's `roofline.traffic` into null.  These
tests pin the arity against the kernel's declaration and, when a committed
profile matches the kernel sources, that every mode's lookup resolves."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _xsmooth_arity():
    src = open(os.path.join(bench.CSRC, "xsmooth.hip")).read()
    m = re.search(r"template\s*<([^>]*)>\s*__global__\s+__launch_bounds__\([^)]*\)\s*void\s+"
                  r"k_xsmooth\(", src)
    assert m, "k_xsmooth declaration not found"
    return len([p for p in m.group(1).split(",") if p.strip()])


def test_kernel_ids_match_the_template_arity():
    n = _xsmooth_arity()
    for (mode, _), names in bench.KERNEL_IDS.items():
        for name in names:
            args = name[name.index("<") + 1:name.rindex(">")].split(",")
            assert len(args) == n, (mode, name, n)


def test_committed_profile_resolves_every_mode():
    sha = bench.kernels_sha()
    import glob
    import json
    modes = {json.load(open(f)).get("mode")
             for f in glob.glob(os.path.join(ROOT, "profiles", "*hbm_traffic*.json"))
             if json.load(open(f)).get("kernel_sources_sha256") == sha}
    if not modes:
        pytest.skip("no committed profile matches the current kernel sources")
    for (mode, _), names in bench.KERNEL_IDS.items():
        if mode not in modes:
            continue
        # (bench keys on the LOADED library's sha; here: the tree's)
        path = None
        for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*hbm_traffic*.json"))):
            d = json.load(open(f))
            if d.get("kernel_sources_sha256") == sha and d.get("mode") == mode:
                path = f
                kernels = d["kernels"]
        assert path
        for kname in names:
            hits = [k for k in kernels if k.split(" grid=")[0] == kname]
            assert hits, (mode, kname, os.path.relpath(path, ROOT))
