"""CPU: the host line scan of the ingest (csrc/wcg_scan.h, Split's P1 rule, mapreduce.go:141-179).

r04 replaced the per-line memchr scan with a windowed memrchr scan; tests/native/ingest_scan_check.cpp
checks that both give the same chunk cut and stop decision through wcg_map_file's caller rule."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")
def test_windowed_scan_matches_per_line_scan(tmp_path):
    exe = tmp_path / "scan_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "mit-6.824-2015_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "ingest_scan_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
