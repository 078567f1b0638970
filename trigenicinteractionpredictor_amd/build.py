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
SRC = os.path.join(PKG, "csrc", "mmsbm.hip")           # triplet engine (include/mmsbm.h)
SRC_PAIRS = os.path.join(PKG, "csrc", "pairs.hip")     # joint model pair lattice (mmsbm_pairs.h)
SRCS = [SRC, SRC_PAIRS]
INCLUDE = os.path.join(REPO, "include")
OUT_DIR = os.path.join(PKG, "_build")
LIB = os.path.join(OUT_DIR, "libmmsbm.so")
SRC_IO = os.path.join(PKG, "csrc", "fold_io.cpp")
LIB_IO = os.path.join(OUT_DIR, "libmmsbm_io.so")  # host-only ingestion (include/mmsbm_io.h)
ARCH = os.environ.get("MMSBM_OFFLOAD_ARCH", "gfx950")
DEPS = {
    SRC: [os.path.join(PKG, "csrc", "plan.h"), os.path.join(PKG, "csrc", "sk.h"),
          os.path.join(INCLUDE, "mmsbm.h")],
    SRC_PAIRS: [os.path.join(INCLUDE, "mmsbm.h"), os.path.join(INCLUDE, "mmsbm_pairs.h")],
}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MMSBM engine needs ROCm's hipcc to build")


def _obj(src: str, out_dir: str = OUT_DIR, tag: str = "") -> str:
    return os.path.join(out_dir, os.path.basename(src).replace(".hip", tag + ".o"))


def compile_command(src: str, obj: str, extra=()) -> list[str]:
    return [hipcc(), "-O3", "-std=c++17", "--offload-arch=" + ARCH, "-fPIC", "-c",
            "-I" + INCLUDE, "-o", obj, src, *extra]


def link_command(out: str, objs) -> list[str]:
    return [hipcc(), "--offload-arch=" + ARCH, "-fPIC", "-shared", "-o", out, *objs]


def command(out: str = LIB, extra=()) -> list[str]:
    """One-shot build of every source into `out` (measurement builds with extra -D flags)."""
    bid_src = _write_build_id(os.path.dirname(os.path.abspath(out)), build_id(extra))
    return [hipcc(), "-O3", "-std=c++17", "--offload-arch=" + ARCH, "-fPIC", "-shared",
            "-I" + INCLUDE, "-o", out, *SRCS, bid_src, *extra]


def build_id(extra=()) -> str:
    """16 hex digits of sha256 over every source and header the library is built from, the
    offload arch and the compile flags: names the build a profile record was taken with
    (bench.py compares it with the loaded library's mmsbm_build_id())."""
    import hashlib
    h = hashlib.sha256()
    files = sorted({f for src in SRCS for f in [src, *DEPS[src]]})
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(["-O3", "-std=c++17", "--offload-arch=" + ARCH, *extra]).encode())
    return h.hexdigest()[:16]


def _write_build_id(out_dir: str, bid: str) -> str:
    """A one-function host source that returns the build id (compiled and linked last)."""
    src = os.path.join(out_dir, "build_id.cpp")
    text = 'extern "C" const char* mmsbm_build_id(void) { return "%s"; }\n' % bid
    if not os.path.exists(src) or open(src).read() != text:
        with open(src, "w") as f:
            f.write(text)
    return src


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def needs_build(out: str = LIB) -> bool:
    return _stale(out, [d for src in SRCS for d in [src, *DEPS[src]]])


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile each source to an object (in parallel, only the stale ones) and link."""
    if not force and not needs_build():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    procs = []
    objs = []
    for src in SRCS:
        obj = _obj(src)
        objs.append(obj)
        if force or _stale(obj, [src, *DEPS[src]]):
            cmd = compile_command(src, obj + ".tmp")
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((subprocess.Popen(cmd), obj))
    for p, obj in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, "hipcc " + obj)
        os.replace(obj + ".tmp", obj)
    bid_obj = os.path.join(OUT_DIR, "build_id.o")
    bid_src = _write_build_id(OUT_DIR, build_id())
    subprocess.check_call([shutil.which("g++") or "g++", "-O2", "-fPIC", "-c", "-o", bid_obj, bid_src])
    objs.append(bid_obj)
    tmp = LIB + ".tmp"
    cmd = link_command(tmp, objs)
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
