"""Lane maps of v_mfma_i32_32x32x32_i8 (gfx950) from exact integer data: which (row, k) of A and (k, col)
of B each lane's 16 bytes hold. Candidate maps are tried against A @ B on the host; the C/D map is the
dtype-independent 32x32 one (cdna_hip_programming.md §3: col = l & 31, row = (r & 3) + 8 (r >> 2) +
4 (l >> 5))."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gadmm_amd.ops import native  # noqa: E402

lib = native.require()
fn = lib.gadmm_mfma_i8_probe
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda", 0)
rng = np.random.default_rng(3)
A = rng.integers(-100, 101, size=(32, 32)).astype(np.int64)
B = rng.integers(-100, 101, size=(32, 32)).astype(np.int64)
ref = A @ B

maps = {
    "k=16h+j": lambda l, j: (l & 31, 16 * (l >> 5) + j),
    "k=8h+j|16+8h+j-8": lambda l, j: (l & 31, (8 * (l >> 5) + j) if j < 8 else (16 + 8 * (l >> 5) + j - 8)),
    "k=4h+j%4+8(j/4)": lambda l, j: (l & 31, 4 * (l >> 5) + (j & 3) + 8 * (j >> 2)),
    "k=2h..": lambda l, j: (l & 31, 2 * (l >> 5) + (j & 1) + 4 * (j >> 1)),
}


def run(mapA, mapB):
    af = np.zeros((64, 16), dtype=np.int8)
    bf = np.zeros((64, 16), dtype=np.int8)
    for l in range(64):
        for j in range(16):
            r, k = mapA(l, j)
            af[l, j] = A[r, k]
            c, k2 = mapB(l, j)
            bf[l, j] = B[k2, c]
    a_t = torch.from_numpy(af.copy()).to(dev)
    b_t = torch.from_numpy(bf.copy()).to(dev)
    d_t = torch.zeros((64 * 16,), dtype=torch.int32, device=dev)
    native.check(fn(a_t.data_ptr(), b_t.data_ptr(), d_t.data_ptr(), None), "probe")
    torch.cuda.synchronize()
    d = d_t.cpu().numpy().reshape(64, 16)
    D = np.zeros((32, 32), dtype=np.int64)
    for l in range(64):
        for r in range(16):
            D[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31] = d[l, r]
    return D


for name, mp in maps.items():
    D = run(mp, mp)
    print("%-22s match=%s" % (name, bool(np.array_equal(D, ref))), flush=True)
