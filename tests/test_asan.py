"""Sanitizer builds: the CPU checker (oracle/mg_oracle.c) and the
host-only multi-GPU partition / exchange plan (csrc/plan.h) compiled with
-fsanitize=address,undefined and run on the CPU; any out-of-bounds access,
leak or undefined behaviour fails the test."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1")


def _run(cmd, exe):
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    _run(["gcc", *SAN, "-ffp-contract=off", "-std=c11", "-I", os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests", "asan", "oracle_asan.c"),
          os.path.join(ROOT, "oracle", "mg_oracle.c"), "-lm", "-o", exe], exe)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_partition_plan_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "plan_asan")
    _run(["g++", *SAN, "-std=c++17", "-I",
          os.path.join(ROOT, "hpcclassmultigridproject_amd", "csrc"),
          os.path.join(ROOT, "tests", "asan", "plan_asan.cpp"), "-o", exe], exe)
