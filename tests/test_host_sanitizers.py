"""Native host runtime under sanitizers.

The CSV encoder, byte-range text shards + tokenizer, SPSC ring, row formatter and checkpoint container are compiled together with a
C++ self-test (avenir_amd/csrc/tests/host_selftest.cpp) twice: with AddressSanitizer +
UndefinedBehaviorSanitizer and with ThreadSanitizer (the ring is exercised by a producer and a
consumer thread, the CSV parser and formatter by 8 worker threads).  GPU-side sanitizers are not
available on the target pool, so device code is covered by the oracle tests instead."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "avenir_amd", "csrc")
SOURCES = [os.path.join(ROOT, "tests", "host_selftest.cpp"), os.path.join(ROOT, "host", "csv.cpp"),
           os.path.join(ROOT, "host", "ring_ckpt.cpp"), os.path.join(ROOT, "host", "records.cpp")]


def _build_and_run(tmp_path, flags: list[str], env_extra: dict[str, str]) -> None:
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-I",
           os.path.join(ROOT, "include"), *flags, *SOURCES, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "OK", (r.stdout[-2000:], r.stderr[-6000:])


def test_host_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0"})


def test_host_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
