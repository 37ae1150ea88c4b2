"""The device formatter's Python-repr routine (``put_repr`` in csrc/kernels/format.hip) compiled
for the HOST from the same source text (g++, __device__ defined away) and compared with Python's
``repr`` on 400 k doubles: random magnitudes 1e-10 .. 1e16, powers of two and their neighbours,
decimal fractions, signed zero and non-finite values.  Values outside the exact 128-bit path must
report "host formatter" (false), never wrong digits.  The GPU twin of this test is
tests/test_format_device.py::test_device_repr_equals_python."""
from __future__ import annotations

import math
import random
import shutil
import struct
import subprocess
from pathlib import Path

import pytest

SRC = Path(__file__).resolve().parents[1] / "avenir_amd" / "csrc" / "kernels" / "format.hip"

HARNESS = r"""
#include <cstdint>
#include <cstdio>
#include <cstring>
#define __device__
#define __forceinline__ inline
static inline long long __double_as_longlong(double v) { long long r; std::memcpy(&r, &v, 8); return r; }
%BODY%
int main() {
  unsigned long long bits;
  char out[64];
  while (std::fread(&bits, 8, 1, stdin) == 1) {
    double v;
    std::memcpy(&v, &bits, 8);
    Sink s{out, 0};
    if (put_repr(s, v)) { std::fwrite(out, 1, (size_t)s.pos, stdout); std::fputc('\n', stdout); }
    else std::fputs("<host>\n", stdout);
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def repr_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    src = SRC.read_text()
    a = src.index("__device__ __forceinline__ int u64_digits")
    b = src.index("__device__ __constant__ uint64_t kPow10")
    c = src.index("__device__ __forceinline__ bool put_repr")
    d = src.index("// [a, e) of field f of the line")
    d_ = tmp_path_factory.mktemp("repr")
    cpp = d_ / "repr.cpp"
    cpp.write_text(HARNESS.replace("%BODY%", src[a:b] + src[c:d]))
    exe = d_ / "repr"
    subprocess.run(["g++", "-O2", "-std=c++17", str(cpp), "-o", str(exe)], check=True)
    return exe


def _values():
    rng = random.Random(5)
    vals = [0.0, -0.0, float("nan"), float("inf"), float("-inf"), 0.1, 0.2, 0.3, 1 / 3, 2 / 3, 1e-4, 1e-5,
            9.999999999999999e-05, 1e15, 123456789.0, 0.5, 2.675, 1.005, 4503599627370496.0, 2251799813685248.5]
    for k in range(-40, 53):
        for s in (1.0, -1.0):
            x = s * math.ldexp(1.0, k)
            vals += [x, math.nextafter(x, 0.0), math.nextafter(x, math.copysign(1e308, x))]
    vals += [i / 1000 for i in range(1, 20000)] + [-i / 7 for i in range(1, 20000)]
    for _ in range(360000):
        vals.append(rng.choice((-1.0, 1.0)) * (0.1 + 9.9 * rng.random()) * 10.0 ** rng.randint(-9, 15))
    return vals


def test_host_build_of_device_repr_equals_python(repr_bin):
    vals = _values()
    data = b"".join(struct.pack("<d", v) for v in vals)
    out = subprocess.run([str(repr_bin)], input=data, capture_output=True, check=True).stdout.decode().split("\n")
    assert len(out) == len(vals) + 1
    for v, got in zip(vals, out):
        if math.isfinite(v) and abs(v) >= 2.0 ** 53:     # the exact path's documented range ends here
            assert got == "<host>", (v, got)
        else:
            assert got == repr(v), (v, got)


def test_out_of_range_values_go_to_the_host(repr_bin):
    vals = [1e300, -2.0 ** 60, 5e-324, 1.2345678901234567e-20]
    data = b"".join(struct.pack("<d", v) for v in vals)
    out = subprocess.run([str(repr_bin)], input=data, capture_output=True, check=True).stdout.decode().split("\n")
    assert out[:4] == ["<host>"] * 4
