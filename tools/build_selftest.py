"""Build the native self-test executable (csrc/tests/native_selftest.cpp + every kernel and runtime
source), plain and with host AddressSanitizer + UndefinedBehaviorSanitizer.

    python tools/build_selftest.py [--asan] [-j 8]      -> build/native_selftest[_asan]

Sanitizer flags apply to host code only (each -fsanitize= follows -Xarch_host; device code is
never instrumented: GPU ASan / XNACK are not used).
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
from gadmm_amd._build import hipcc, ARCH  # noqa: E402

CSRC = os.path.join(ROOT, "csrc")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]


def build(asan: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    tag = "asan" if asan else "plain"
    obj_dir = os.path.join(ROOT, "build", "selftest_" + tag)
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
                  + [os.path.join(CSRC, "tests", "native_selftest.cpp")])
    hdrs = glob.glob(os.path.join(CSRC, "include", "*.h"))
    extra = SAN if asan else []
    opt = ["-O3"]  # device code is never instrumented; keep its codegen identical to the library

    def one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in hdrs])
        if os.path.exists(obj) and os.path.getmtime(obj) >= dep:
            return obj
        cmd = [hipcc(), "-c", src, "-o", obj, "-fPIC", "-std=c++17", "-I", os.path.join(CSRC, "include")] + opt + extra
        if src.endswith(".hip"):
            cmd += ["--offload-arch=%s" % ARCH, "-x", "hip", "-munsafe-fp-atomics"]
        else:
            cmd += ["-D__HIP_PLATFORM_AMD__"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
        return obj

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(one, srcs))
    exe = os.path.join(ROOT, "build", "native_selftest" + ("_asan" if asan else ""))
    cmd = [hipcc(), "-o", exe] + objs + ["--offload-arch=%s" % ARCH, "-lrccl", "-lamdhip64"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
    if verbose:
        print("built", exe)
    return exe


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--asan", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    build(a.asan, a.j)
