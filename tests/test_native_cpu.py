"""Native library: builds for gfx950 here (no GPU) and its C ABI matches the ctypes mirrors."""
import ctypes
import os

from gadmm_amd import _build
from gadmm_amd.ops import native


def test_builds_and_loads():
    lib_path = _build.build(verbose=False)
    assert os.path.exists(lib_path)
    assert native.available()
    lib = native.require()
    assert lib.gadmm_native_version() >= 1
    assert lib.gadmm_rccl_version() >= 22000


def test_abi_layout_matches_ctypes():
    lib = native.require()
    fn = lib.gadmm_abi_layout
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = (ctypes.c_longlong * 32)()
    k = fn(buf, 32)
    got = list(buf[:k])
    exp = [ctypes.sizeof(native.PhaseSlot), ctypes.sizeof(native.XchgOp), ctypes.sizeof(native.ChainCtl),
           ctypes.sizeof(native.PhaseArgs), native.PhaseArgs.rho.offset, native.PhaseArgs.ring.offset,
           native.PhaseArgs.inner_iters.offset, ctypes.sizeof(native.EngineDesc), native.EngineDesc.stream.offset,
           ctypes.sizeof(native.RunStats), ctypes.sizeof(native.PersistArgs), native.PersistArgs.rho.offset,
           native.PersistArgs.ctl.offset]
    assert got == exp


def test_fo_abi_layout_matches_ctypes():
    lib = native.require()
    buf = (ctypes.c_longlong * 16)()
    k = lib.gadmm_fo_abi_layout(buf, 16)
    exp = [ctypes.sizeof(native.FoCtl), ctypes.sizeof(native.FoArgs), native.FoArgs.step.offset,
           native.FoArgs.timeout_ticks.offset, native.FoArgs.A.offset, native.FoArgs.ctl.offset]
    assert list(buf[:k]) == exp


def test_code_objects_target_gfx950():
    import subprocess
    lib = native.library_path()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib], capture_output=True,
                         text=True)
    txt = out.stdout + out.stderr
    assert "gfx950" in txt
