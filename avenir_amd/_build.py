"""Native build for avenir_amd: hand-written HIP/CDNA4 kernels + host C++ runtime.

Everything is compiled IN-TREE into ``avenir_amd/_C.so`` (one Python extension module):

* ``csrc/kernels/*.hip``  -> ``hipcc --offload-arch=gfx950`` device code.  These translation units
  include no torch headers, so they compile in seconds.
* ``csrc/host/*.cpp``     -> host-only C++ runtime (CSV->columnar parser, config, ring buffer,
  checkpoint container).  Compiled with the same clang driver, no offload.
* ``csrc/bindings.cpp`` + ``csrc/bind_*.cpp`` -> the only TUs that include torch / pybind11.

A ``build.ninja`` file is generated so rebuilds are incremental and parallel.  Run
``python -m avenir_amd._build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
OUT = PKG / "_C.so"
ARCH = os.environ.get("AVENIR_ARCH", "gfx950")


def _torch_paths():
    import torch
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return inc, tdir / "lib"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found; the ROCm toolchain is required to build avenir_amd")


def sources():
    kern = sorted((CSRC / "kernels").glob("*.hip"))
    host = sorted((CSRC / "host").glob("*.cpp"))
    return kern, host, [CSRC / "bindings.cpp"] + sorted(CSRC.glob("bind_*.cpp"))


def write_ninja(debug: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    tinc, tlib = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    opt = "-O0 -g" if debug else "-O3"
    common = f"{opt} -fPIC -std=c++17 -I{CSRC / 'include'} -Wno-unused-result -Wno-deprecated-declarations"
    kflags = (f"{common} --offload-arch={ARCH} -munsafe-fp-atomics "
              "-D__HIP_PLATFORM_AMD__=1")
    rocm_inc = "-isystem /opt/rocm/include"
    hflags = f"{common} {rocm_inc} -D__HIP_PLATFORM_AMD__=1 -pthread -march=x86-64-v3"
    bflags = (f"{common} {rocm_inc} -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_C "
              f"-DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI=1 "
              + " ".join(f"-isystem {p}" for p in tinc) + f" -isystem {pyinc}")
    libs = (f"-L{tlib} -Wl,-rpath,{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip "
            f"-ltorch_python -lamdhip64 -pthread")
    kern, host, bind = sources()
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"kflags = {kflags}",
        f"hflags = {hflags}",
        f"bflags = {bflags}",
        f"libs = {libs}",
        "rule kcc",
        "  command = $hipcc $kflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule hcc",
        "  command = $hipcc -x c++ $hflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule bcc",
        "  command = $hipcc -x c++ $bflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = BIND $in",
        "rule link",
        "  command = $hipcc --offload-arch=" + ARCH + " -shared -fPIC $in -o $out $libs",
        "  description = LINK $out",
    ]
    objs = []
    for s in kern:
        o = BUILD / (s.stem + ".hip.o")
        lines.append(f"build {o}: kcc {s}")
        objs.append(o)
    for s in host:
        o = BUILD / (s.stem + ".host.o")
        lines.append(f"build {o}: hcc {s}")
        objs.append(o)
    for s in bind:
        ob = BUILD / (s.stem + ".o")
        lines.append(f"build {ob}: bcc {s}")
        objs.append(ob)
    lines.append(f"build {OUT}: link " + " ".join(str(o) for o in objs))
    lines.append(f"default {OUT}")
    nf = BUILD / "build.ninja"
    txt = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != txt:
        nf.write_text(txt)
    return nf


def build(debug: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    nf = write_ninja(debug)
    ninja = shutil.which("ninja")
    if ninja is None:
        try:
            import ninja as _nj  # type: ignore
            ninja = str(Path(_nj.BIN_DIR) / "ninja")
        except Exception as exc:  # pragma: no cover
            raise RuntimeError("ninja is required to build avenir_amd") from exc
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [ninja, "-f", str(nf), "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=str(BUILD))
    return OUT


if __name__ == "__main__":
    build(debug="--debug" in sys.argv, verbose="-v" in sys.argv)
    print(f"built {OUT}")
