"""Build ``gadmm_amd/_native/libgadmm_native.so`` for gfx950 (MI355X) with hipcc.

The native library is plain HIP C++ with a C ABI (no torch headers): kernels under ``csrc/kernels``
and the runtime (chain engine, RCCL communicator) under ``csrc/runtime``. It is built in-tree so it
travels with the repository snapshot to the GPU box. Incremental: a translation unit is recompiled
only when it or a header is newer than its object file.

    python -m gadmm_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "gadmm_amd", "_native")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(OUT_DIR, "libgadmm_native.so")
ARCH = os.environ.get("GADMM_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build gadmm_amd native code)")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "include", "*.h")))


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(OBJ_DIR, rel + ".o")


def _compile(src: str, force: bool) -> str:
    obj = _obj_for(src)
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [hipcc(), "-c", src, "-o", obj, "-fPIC", "-O3", "-std=c++17", "-I", os.path.join(CSRC, "include"),
           "-Wno-unused-result"]
    if src.endswith(".hip"):
        cmd += ["--offload-arch=%s" % ARCH, "-x", "hip", "-munsafe-fp-atomics"]
    else:
        cmd += ["-D__HIP_PLATFORM_AMD__"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr))
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    srcs = sources()
    if not force and os.path.exists(LIB) and \
            os.path.getmtime(LIB) >= max(os.path.getmtime(p) for p in srcs + headers()):
        # the library is newer than every source and header: up to date without looking at objects. The
        # GPU box receives the library but not build/ (.gpurunignore), and without this check every
        # process there re-ran the toolchain on its first native call (~5 s, profiles/r06_entries)
        if verbose:
            print("up to date", LIB)
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        cmd = [hipcc(), "-shared", "-o", LIB + ".tmp"] + objs + [
            "--offload-arch=%s" % ARCH, "-L", os.path.join(rocm, "lib"), "-lrccl", "-lamdhip64"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr))
        os.replace(LIB + ".tmp", LIB)
        if verbose:
            print("built", LIB)
    elif verbose:
        print("up to date", LIB)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
