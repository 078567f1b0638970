"""Build libmmsbm.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The shared object lands in trigenicinteractionpredictor_amd/_build/ so it
travels with the repository snapshot to the GPU box (it is git-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "mmsbm.hip")
INCLUDE = os.path.join(REPO, "include")
OUT_DIR = os.path.join(PKG, "_build")
LIB = os.path.join(OUT_DIR, "libmmsbm.so")
SRC_IO = os.path.join(PKG, "csrc", "fold_io.cpp")
LIB_IO = os.path.join(OUT_DIR, "libmmsbm_io.so")  # host-only ingestion (include/mmsbm_io.h)
ARCH = os.environ.get("MMSBM_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MMSBM engine needs ROCm's hipcc to build")


def command(out: str = LIB, extra=()) -> list[str]:
    return [hipcc(), "-O3", "-std=c++17", "--offload-arch=" + ARCH, "-fPIC", "-shared",
            "-I" + INCLUDE, "-o", out, SRC, *extra]


def needs_build(out: str = LIB) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [SRC, os.path.join(PKG, "csrc", "plan.h"), os.path.join(INCLUDE, "mmsbm.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = command(tmp)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


def build_io(force: bool = False, verbose: bool = True) -> str:
    """Host C++ fold reader (no GPU code): g++ -O2."""
    deps = [SRC_IO, os.path.join(INCLUDE, "mmsbm_io.h")]
    if not force and os.path.exists(LIB_IO) and all(os.path.getmtime(d) <= os.path.getmtime(LIB_IO)
                                                     for d in deps):
        return LIB_IO
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB_IO + ".tmp"
    cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I" + INCLUDE,
           "-o", tmp, SRC_IO]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB_IO)
    return LIB_IO


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_io(force="--force" in sys.argv)
