"""CPU: bench.py's N > 1 watchdog (bench.Watchdog) turns a phase that waits
on peers past its deadline -- an RCCL hang -- into one error JSON line and
exit status 1, instead of a run that stalls until an outer time limit."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench
with bench.Watchdog("rccl_selfcheck", {secs}, rank=3, world=8):
    time.sleep({sleep})
print("phase finished", flush=True)
"""


def _run(secs, sleep):
    code = _CHILD.format(root=ROOT, secs=secs, sleep=sleep)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=60)


def test_watchdog_fires_with_an_error_line_and_status_1():
    r = _run(0.5, 30)
    assert r.returncode == 1, (r.returncode, r.stdout, r.stderr)
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and line["n_gpus"] == 8
    assert "rccl_selfcheck" in line["error"] and "rank 3" in line["error"]


def test_watchdog_quiet_when_the_phase_finishes():
    r = _run(20, 0.1)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "phase finished"


def test_watchdog_off_for_one_gpu():
    code = _CHILD.format(root=ROOT, secs=0.2, sleep=1.0).replace("world=8", "world=1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "phase finished"
