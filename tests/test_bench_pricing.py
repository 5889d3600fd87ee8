"""CPU: the (dist_min_rows, dist_overlap) pairs bench.py's N > 1 warm-up
prices (bench.pricing_candidates): the set itself, and that a pair the RCCL
self-check did not pass bitwise is never timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _check(fail=(), base_fail=()):
    """A self-check verdict: min_rows 16 per overlap, candidates per pair."""
    modes = {str(ov): {"passed": str(ov) not in base_fail} for ov in (0, 1, 2)}
    cand = {f"{r}:{ov}": {"passed": f"{r}:{ov}" not in fail}
            for r in (128, 256, 512) for ov in (0, 1, 2)}
    return {"modes": modes, "candidates": cand}


def test_candidate_set_at_the_headline_size():
    c = bench.pricing_candidates("auto", "auto", 16384, None)
    assert c == [(r, ov) for r in (128, 256, 512) for ov in (0, 1, 2)]
    # the rows the self-check must cover are exactly these
    assert sorted({r for r, _ in c}) == list(bench.MIN_ROWS_CANDIDATES)


def test_above_headline_size_only_the_default_rows():
    c = bench.pricing_candidates("auto", "auto", 65536, None)
    assert c == [(256, 0), (256, 1), (256, 2)]


def test_fixed_arguments():
    assert bench.pricing_candidates("1", "128", 16384, None) == [(128, 1)]
    assert bench.pricing_candidates("auto", "256", 16384, None) == [(256, 0), (256, 1), (256, 2)]


def test_failed_self_check_pairs_are_dropped():
    c = bench.pricing_candidates("auto", "auto", 16384, _check(fail=("128:2", "256:0")))
    assert (128, 2) not in c and (256, 0) not in c and len(c) == 7
    # an overlap mode whose min_rows 16 check failed is dropped for every rows value
    c = bench.pricing_candidates("auto", "auto", 16384, _check(base_fail=("1",)))
    assert all(ov != 1 for _, ov in c) and len(c) == 6


def test_never_empty():
    every = tuple(f"{r}:{ov}" for r in (128, 256, 512) for ov in (0, 1, 2))
    assert bench.pricing_candidates("auto", "auto", 16384, _check(fail=every)) == [(256, 0)]
