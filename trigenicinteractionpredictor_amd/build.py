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
    deps = [SRC, os.path.join(INCLUDE, "mmsbm.h")]
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


if __name__ == "__main__":
    build(force="--force" in sys.argv)
