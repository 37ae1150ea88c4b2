"""The shared decimal parser (csrc/include/avenir_numparse.h: Clinger fast path + Eisel-Lemire,
ADVICE r4) against the C library's correctly rounded strtod, compiled as a host program: ~1.5 M
tokens, zero mismatches allowed."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "avenir_amd" / "csrc" / "tests" / "numparse_check.cpp"


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_numparse_matches_strtod(tmp_path):
    exe = tmp_path / "numparse_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "avenir_amd" / "csrc" / "include"), str(SRC),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " bad 0 " in r.stdout, r.stdout
