"""Time the symmetric-GEMV variants of tools/symv_lab.hip at d = 10000 (real10m's packed inverses):
python tools/symv_lab.py [d] [reps]. Prints one line per variant: us per GEMV, effective TB/s of the
packed matrix, max relative difference against variant 0 (and v0 against torch)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsymv_lab.so"))
    lib.symv_lab_time.restype = ctypes.c_double
    lib.symv_lab_time.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3
    for f in ("symv_lab_packed_doubles", "symv_lab_part_doubles", "symv_lab_padded"):
        getattr(lib, f).restype = ctypes.c_long
        getattr(lib, f).argtypes = [ctypes.c_int]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    full = torch.randn(d, d, dtype=torch.float64, device=dev, generator=g)
    full = full + full.T
    from gadmm_amd.ops.linalg import sym_pack
    Mp = sym_pack(full.unsqueeze(0))[0].contiguous()
    assert Mp.numel() == lib.symv_lab_packed_doubles(d)
    r = torch.zeros(lib.symv_lab_padded(d), dtype=torch.float64, device=dev)
    r[:d] = torch.randn(d, dtype=torch.float64, device=dev, generator=g)
    ref = full @ r[:d]
    del full
    torch.cuda.synchronize()
    P = torch.zeros(lib.symv_lab_part_doubles(d), dtype=torch.float64, device=dev)
    nbytes = Mp.numel() * 8
    y0 = None
    print("d=%d packed=%.1f MB" % (d, nbytes / 1e6), flush=True)
    for v, k in ((0, 0), (1, 0), (2, 0), (3, 4), (3, 8), (4, 0), (9, 8), (9, 32)):
        y = torch.zeros(lib.symv_lab_padded(d), dtype=torch.float64, device=dev)
        us = lib.symv_lab_time(v, Mp.data_ptr(), r.data_ptr(), P.data_ptr(), y.data_ptr(), d, k, reps)
        torch.cuda.synchronize()
        line = "v%d k=%d  %.1f us  %.2f TB/s" % (v, k, us, nbytes / (us * 1e-6) / 1e12)
        if v != 9:
            yy = y[:d].clone()
            if y0 is None:
                y0 = yy
                line += "  vs torch %.2e" % float((yy - ref).abs().max() / ref.abs().max())
            else:
                line += "  vs v0 %.2e" % float((yy - y0).abs().max() / y0.abs().max())
        print(line, flush=True)


if __name__ == "__main__":
    main()
