"""Dense f64 linear-algebra ops with a HIP path (gfx950) and a PyTorch CPU path.

* ``gram(X, y)``: per-worker ``A = X^T X``, ``b = X^T y``, ``yy = y^T y`` (kernel K1: one f64-MFMA
  SYRK of the augmented shard ``[X | y]``, csrc/kernels/gram.hip).
* ``spd_inverse(A, shifts)``: ``(A_n + s_{n,v} I)^{-1}`` for every worker n and shift v
  (kernel K2: in-LDS Gauss-Jordan for d <= 128, csrc/kernels/spd_inverse.hip; blocked Gauss-Jordan
  with f64-MFMA rank-128 updates for larger d, csrc/kernels/spd_inverse_blocked.hip. One-time set-up;
  ``GADMM_BIGINV=rocsolver`` selects torch's Cholesky + cholesky_inverse instead, for A/B runs).

CUDA tensors always take the native path (and raise if the library is missing); CPU tensors use
torch, which is also the fp64 reference the kernels are tested against.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import native
from ..utils.env import getenv


def gram_torch(X: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    Xt = X.transpose(1, 2)
    A = torch.bmm(Xt, X)
    b = torch.bmm(Xt, y.unsqueeze(-1)).squeeze(-1)
    yy = (y * y).sum(dim=1)
    return A, b, yy


# The int8 schemes (Ozaki digits, CRT) keep 49 bits of every value relative to its column's scale (>= the column maximum), so
# an entry at the column's rms level keeps ~49 - log2(colmax / rms) bits; past 2^4 (45 bits, against the
# 53 of an f64 operand) ``gram`` recomputes the shard on the f64-MFMA kernel. Gaussian columns of a
# million rows sit near 5; one outlier row, or a heavy-tailed (e.g. lognormal) column, exceeds it.
OZ_MAX_RANGE = 16.0
LAST_GRAM: dict = {}  # path of the last CUDA ``gram`` call (``path``, ``range``): benchmarks report it


def gram_ozaki(X: torch.Tensor, y: torch.Tensor, out=None, with_range: bool = False):
    """Batched augmented Gram on the INT8 matrix cores (csrc/kernels/gram_ozaki.hip: the Ozaki scheme --
    7 int8 digits per f64 value after a per-column power-of-two scaling, exact int32 MFMA products of the
    28 digit pairs that reach f64 precision, f64 recombination). Same outputs as ``gram``; not bit-equal
    to the f64-MFMA Gram (a different, exactly summed evaluation). ``with_range``: also return each
    shard's column-range statistic max_j colmax_j / rms_j (an (N,) device tensor; the accuracy gate of
    ``gram``). The workspace (about 2.0 GB at d = 10k: the padded f64 Gram 0.82 GB + two digit chunks
    1.16 GB) is taken from torch's caching allocator per call and returned after it, not held."""
    lib = native.require()
    X = X.contiguous()
    y = y.contiguous()
    N, m, d = X.shape
    if out is not None:
        A, b, yy = out
    else:
        A = torch.empty((N, d, d), dtype=torch.float64, device=X.device)
        b = torch.empty((N, d), dtype=torch.float64, device=X.device)
        yy = torch.empty((N,), dtype=torch.float64, device=X.device)
    rng = torch.empty((N,), dtype=torch.float64, device=X.device)
    nb = int(lib.gadmm_gram_ozaki_workspace(int(m), int(d)))
    ws = torch.empty((nb,), dtype=torch.uint8, device=X.device)
    native.check(lib.gadmm_gram_ozaki_f64(X.data_ptr(), y.data_ptr(), int(N), int(m), int(d), A.data_ptr(),
                                          b.data_ptr(), yy.data_ptr(), ws.data_ptr(), nb, rng.data_ptr(),
                                          native.stream_handle()),
                 "gram_ozaki_f64")
    del ws  # back to the caching allocator once the stream has used it (stream-ordered reuse)
    return (A, b, yy, rng) if with_range else (A, b, yy)


def gram_crt(X: torch.Tensor, y: torch.Tensor, out=None, with_range: bool = False):
    """Batched augmented Gram on the INT8 matrix cores by CRT slicing (csrc/kernels/gram_crt.hip: 49-bit
    integer images of the column-scaled values, one int8 GEMM with exact int32 sums per modulus for 16
    coprime moduli <= 234, Garner reconstruction of the exact integer Gram, one final rounding). Same
    outputs and accuracy class as ``gram_ozaki`` (the digit scheme keeps the same 49 bits); one accumulator
    per output element instead of seven, so 256 x 256 tiles. m <= 2^21 rows per shard. ``with_range``:
    also the (N,) column-range statistics of the accuracy gate."""
    lib = native.require()
    X = X.contiguous()
    y = y.contiguous()
    N, m, d = X.shape
    if m > int(lib.gadmm_gram_crt_max_rows()):
        raise ValueError("gram_crt: %d rows per shard exceed the exact-reconstruction bound" % m)
    if out is not None:
        A, b, yy = out
    else:
        A = torch.empty((N, d, d), dtype=torch.float64, device=X.device)
        b = torch.empty((N, d), dtype=torch.float64, device=X.device)
        yy = torch.empty((N,), dtype=torch.float64, device=X.device)
    rng = torch.empty((N,), dtype=torch.float64, device=X.device)
    nb = int(lib.gadmm_gram_crt_workspace(int(m), int(d)))
    ws = torch.empty((nb,), dtype=torch.uint8, device=X.device)
    native.check(lib.gadmm_gram_crt_f64(X.data_ptr(), y.data_ptr(), int(N), int(m), int(d), A.data_ptr(),
                                        b.data_ptr(), yy.data_ptr(), ws.data_ptr(), nb, rng.data_ptr(),
                                        native.stream_handle()), "gram_crt_f64")
    del ws
    return (A, b, yy, rng) if with_range else (A, b, yy)


def gram_uses_ozaki(m: int, d: int) -> bool:
    """Whether ``gram`` takes an int8 matrix-core path. ``GADMM_GRAM_OZAKI``: ``auto`` (default) for shards
    where the selected scheme measured faster than the f64-MFMA Gram -- the CRT scheme from d >= 1024 and
    m d >= 2^26 (profiles/r06_crt, profiles/r06_dgadmm/crt_small.log), the digit scheme from d >= 3072 and
    m >= 65536 (1.11x at 100k x 4096, 1.10x at 312k x 10k: profiles/r05_h); ``1`` for every d > 256; ``0``
    never. The range gate (``OZ_MAX_RANGE``) applies to both schemes."""
    mode = getenv("GADMM_GRAM_OZAKI", "auto")
    if mode == "0":
        return False
    if mode == "1":
        return d > 256
    if gram_int8_scheme(m) == "crt":
        # measured crossover of the CRT kernel against the f64-MFMA Gram (profiles/r06_dgadmm/crt_small.log):
        # faster at 65k x 1024 (2.3 vs 2.5 ms), 33k x 2048, 20k x 4096; slower at 262k x 512 (4.6 vs 3.1)
        return d >= 1024 and m * d >= (1 << 26)
    return d >= 3072 and m >= 65536


def gram_int8_scheme(m: int) -> str:
    """``crt`` (csrc/kernels/gram_crt.hip, default) or ``digits`` (gram_ozaki.hip). ``GADMM_GRAM_INT8``
    forces one; the CRT reconstruction bound caps it at 2^21 rows per shard, past which the digits run."""
    mode = getenv("GADMM_GRAM_INT8", "crt")
    if mode == "digits":
        return "digits"
    return "crt" if m <= _crt_max_rows() else "digits"


def _crt_max_rows() -> int:
    return int(native.require().gadmm_gram_crt_max_rows())


def gram(X: torch.Tensor, y: torch.Tensor, ksplit: Optional[int] = None, out=None
         ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Batched augmented Gram. ``X``: (N, m, d) f64 contiguous, ``y``: (N, m).
    ``out``: optional preallocated ``(A, b, yy)`` written in place. Large shards go to the int8 matrix
    cores (``gram_crt``, or ``gram_ozaki`` past its row bound or when the CRT workspace -- ~14 GB at
    d = 10k -- cannot be allocated). Shards that path would serve with fewer kept bits than
    ``OZ_MAX_RANGE`` allows (an outlier row, a heavy-tailed column) are recomputed on the f64-MFMA kernel
    (one host read of the N range statistics: set-up code, never graph-captured)."""
    if X.dtype != torch.float64 or y.dtype != torch.float64:
        raise TypeError("gram expects float64")
    if X.is_cuda and ksplit is None and gram_uses_ozaki(int(X.shape[1]), int(X.shape[2])):
        scheme = gram_int8_scheme(int(X.shape[1]))
        res = None
        if scheme == "crt":
            try:
                res = gram_crt(X, y, out=out, with_range=True)
            except torch.cuda.OutOfMemoryError:
                scheme = "digits"
        if res is None:
            res = gram_ozaki(X, y, out=out, with_range=True)
        A, b, yy, rng = res
        r = float(rng.max().item())
        limit = float(getenv("GADMM_OZ_MAX_RANGE", str(OZ_MAX_RANGE)))
        name = "crt-int8" if scheme == "crt" else "ozaki-int8"
        if r <= limit:
            LAST_GRAM.update(path=name, range=r)
            return A, b, yy
        LAST_GRAM.update(path="f64-mfma (%s range gate: %.3g > %g)" % (name, r, limit), range=r)
        return _gram_f64(X, y, None, (A, b, yy))
    if not X.is_cuda:
        res = gram_torch(X, y)
        if out is not None:
            for o, r in zip(out, res):
                o.copy_(r)
            return out
        return res
    LAST_GRAM.update(path="f64-mfma", range=None)
    return _gram_f64(X, y, ksplit, out)


def _gram_f64(X, y, ksplit, out):
    lib = native.require()
    X = X.contiguous()
    y = y.contiguous()
    N, m, d = X.shape
    if out is not None:
        A, b, yy = out
    else:
        A = torch.empty((N, d, d), dtype=torch.float64, device=X.device)
        b = torch.empty((N, d), dtype=torch.float64, device=X.device)
        yy = torch.empty((N,), dtype=torch.float64, device=X.device)
    if ksplit is None:
        ksplit = int(lib.gadmm_gram_pick_ksplit(N, m, d))
    ws_n = int(lib.gadmm_gram_workspace(N, m, d, ksplit))
    ws = torch.empty((max(ws_n, 1),), dtype=torch.float64, device=X.device) if ws_n > 0 else None
    rc = lib.gadmm_gram_f64(X.data_ptr(), y.data_ptr(), N, m, d, ksplit, A.data_ptr(), b.data_ptr(),
                            yy.data_ptr(), ws.data_ptr() if ws is not None else None, native.stream_handle())
    native.check(rc, "gram_f64")
    return A, b, yy


def spd_inverse_torch(A: torch.Tensor, shifts: torch.Tensor) -> torch.Tensor:
    N, d, _ = A.shape
    V = shifts.shape[1]
    eye = torch.eye(d, dtype=A.dtype, device=A.device)
    M = A.unsqueeze(1) + shifts.to(A.dtype).view(N, V, 1, 1) * eye
    L = torch.linalg.cholesky(M.reshape(N * V, d, d))
    inv = torch.cholesky_inverse(L)
    inv = 0.5 * (inv + inv.transpose(-1, -2))
    return inv.reshape(N, V, d, d)


def spd_inverse(A: torch.Tensor, shifts: torch.Tensor, out: Optional[torch.Tensor] = None,
                check_status: bool = True, status: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``(N, V, d, d)`` inverses of ``A_n + shifts[n, v] I`` (all SPD); ``out`` written in place.
    ``status``: optional preallocated int32 word (the not-SPD flag; sticky once set)."""
    shifts = torch.as_tensor(shifts, dtype=torch.float64, device=A.device)
    if shifts.dim() == 1:
        shifts = shifts.unsqueeze(0).expand(A.shape[0], -1)
    if not shifts.is_contiguous():
        shifts = shifts.contiguous()
    N, d, _ = A.shape
    V = shifts.shape[1]
    if A.is_cuda and d > 128 and getenv("GADMM_BIGINV", "native") != "rocsolver":
        return spd_inverse_blocked(A, shifts, out=out, check_status=check_status, status=status)
    if not A.is_cuda or d > 128:
        res = spd_inverse_torch(A, shifts)
        if out is not None:
            out.copy_(res)
            return out
        return res
    lib = native.require()
    if out is None:
        out = torch.empty((N, V, d, d), dtype=torch.float64, device=A.device)
    if status is None:
        status = torch.zeros((1,), dtype=torch.int32, device=A.device)
    rc = lib.gadmm_spd_inverse_small_f64(A.contiguous().data_ptr(), shifts.data_ptr(), N, d, V, out.data_ptr(),
                                         status.data_ptr(), native.stream_handle())
    native.check(rc, "spd_inverse_small_f64")
    if check_status and int(status.item()) != 0:
        raise FloatingPointError("spd_inverse: matrix is not positive definite")
    return out


def spd_inverse_blocked(A: torch.Tensor, shifts: torch.Tensor, out: Optional[torch.Tensor] = None, nb: int = 128,
                        check_status: bool = True, status: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Large-d ``(N, V, d, d)`` inverses of ``A_n + shifts[n, v] I`` on the device: blocked in-place
    Gauss-Jordan, f64-MFMA rank-``nb`` updates (csrc/kernels/spd_inverse_blocked.hip)."""
    lib = native.require()
    shifts = torch.as_tensor(shifts, dtype=torch.float64)
    if shifts.dim() == 1:
        shifts = shifts.unsqueeze(0).expand(A.shape[0], -1)
    N, d, _ = A.shape
    V = shifts.shape[1]
    sh = shifts.detach().to("cpu", torch.float64).contiguous()  # set-up: scalars by value per launch
    if out is None:
        out = torch.empty((N, V, d, d), dtype=torch.float64, device=A.device)
    ws = torch.zeros((int(lib.gadmm_spd_inverse_blocked_workspace(d, nb)),), dtype=torch.float64, device=A.device)
    if status is None:
        status = torch.zeros((1,), dtype=torch.int32, device=A.device)
    rc = lib.gadmm_spd_inverse_blocked_f64(A.contiguous().data_ptr(), sh.data_ptr(), N, d, V, out.data_ptr(),
                                           ws.data_ptr(), status.data_ptr(), nb, native.stream_handle())
    native.check(rc, "spd_inverse_blocked_f64")
    if check_status and int(status.item()) != 0:
        raise FloatingPointError("spd_inverse: matrix is not positive definite")
    return out


def sym_pack(M: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Block-packed lower triangles (csrc/include/sym_gemv.h) of the symmetric matrices ``M`` (..., d, d):
    returns (count, packed_doubles(d)) f64 on M's device (the large-d kernels' cached inverses: half
    the bytes an iteration streams)."""
    lib = native.require()
    d = int(M.shape[-1])
    cnt = int(M.numel() // (d * d))
    n = int(lib.gadmm_sym_packed_doubles(d))
    if out is None:
        out = torch.empty((cnt, n), dtype=torch.float64, device=M.device)
    Mc = M.contiguous()
    native.check(lib.gadmm_sym_pack_f64(Mc.data_ptr(), out.data_ptr(), cnt, d, native.stream_handle()), "sym_pack")
    return out


def symv_packed(Mp: torch.Tensor, x: torch.Tensor, out: torch.Tensor, work: torch.Tensor, d: int) -> torch.Tensor:
    """``out = M x`` for ONE block-packed symmetric matrix (``sym_pack``) on the current stream: the
    symmetric GEMV of the large-d engines (csrc/kernels/first_order_big.hip: gadmm_symv_batch, one read
    of each stored block for both products, fixed-order reduction). ``x`` / ``out`` are zero padded to
    ``sym_padded(d)`` (only out[:d] is written); ``work``: ``symv_work_doubles(d)`` doubles."""
    lib = native.require()
    fn = lib.gadmm_symv_batch
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    native.check(fn(Mp.data_ptr(), 0, x.data_ptr(), 0, out.data_ptr(), 0, work.data_ptr(), 1, int(d), None,
                    native.stream_handle()), "symv_batch")
    return out


def sym_padded(d: int) -> int:
    """Length of a vector zero padded for the block-packed symmetric GEMV (sym_gemv.h)."""
    lib = native.require()
    lib.gadmm_sym_padded.restype = ctypes.c_long
    lib.gadmm_sym_padded.argtypes = [ctypes.c_int]
    return int(lib.gadmm_sym_padded(int(d)))


def symv_work_doubles(d: int) -> int:
    lib = native.require()
    lib.gadmm_symv_work_doubles.restype = ctypes.c_long
    lib.gadmm_symv_work_doubles.argtypes = [ctypes.c_int]
    return int(lib.gadmm_symv_work_doubles(int(d)))


def sym_unpack_torch(P: torch.Tensor, d: int, B: int = 128) -> torch.Tensor:
    """The full symmetric matrices of block-packed lower triangles (reference / tests)."""
    nb = (d + B - 1) // B
    out = torch.zeros((P.shape[0], nb * B, nb * B), dtype=P.dtype, device=P.device)
    b = 0
    for i in range(nb):
        for j in range(i + 1):
            blk = P[:, b * B * B:(b + 1) * B * B].reshape(-1, B, B)
            out[:, i * B:(i + 1) * B, j * B:(j + 1) * B] = blk
            if i != j:
                out[:, j * B:(j + 1) * B, i * B:(i + 1) * B] = blk.transpose(1, 2)
            b += 1
    return out[:, :d, :d]


def gemm_f64(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """``A @ B`` (row-major f64) with the MFMA tile kernel of the blocked inverse (tests)."""
    lib = native.require()
    A, B = A.contiguous(), B.contiguous()
    C = torch.empty((A.shape[0], B.shape[1]), dtype=torch.float64, device=A.device)
    native.check(lib.gadmm_gemm_f64_test(A.shape[0], B.shape[1], A.shape[1], A.data_ptr(), B.data_ptr(),
                                         C.data_ptr(), native.stream_handle()), "gemm_f64_test")
    return C
