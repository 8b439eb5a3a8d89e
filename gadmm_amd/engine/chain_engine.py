"""Python front-end of the native chain engine (csrc/runtime/chain_engine.cpp).

One instance per rank. It owns the device state of the rank's logical workers:

* ``theta``  (N_total, d)  primal table; rows of local workers are authoritative, other rows are
  ghost copies of chain neighbours refreshed by the RCCL exchange;
* ``mu``     (N_local, d)  per-worker aggregated duals (D-GADMM form, == edge duals of GADMM);
* linear model: Gram ``A`` (N_local, d, d), ``b``, ``yy`` and the cached inverses
  ``(A + c rho I)^{-1}`` for chain degree c in {1, 2};
* logistic model: the shards themselves (inner GD reads them every step);
* ``ctl`` (ChainCtl), the objective ``trace`` and the multi-rank partial-objective ring.

The iteration loop itself runs in C++ (graph-captured kernels + RCCL), so a solve is one call.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops import native
from ..utils import timing as _timing
from ..ops.linalg import gram, spd_inverse, sym_pack
from ..parallel.topology import Placement, chain_plan, RankPlan
from ..utils.env import getenv


class ResidencyError(RuntimeError):
    """A persistent kernel's workgroups cannot all be resident on this device at once."""


class HandoffTimeout(RuntimeError):
    """A persistent kernel's hand-off spin passed its deadline (done == 4) on some workgroup."""


@dataclass
class EngineRun:
    iters: int
    done: int
    iterations_launched: int
    replays: int
    wall_ms: float
    p2p_bytes: int
    p2p_msgs: int
    monitor_bytes: int
    wire_bytes: int = 0

    @property
    def converged(self) -> bool:
        return self.done == 1


def epoch_tables_numpy(P: np.ndarray, loc: np.ndarray):
    """Per-epoch (slots (E, n_local, 4) = (li, gid, left, right), positions (E, n_local)) of the local
    workers ``loc`` for chains ``P`` (E, n) position -> worker: the reference for the native
    ``gadmm_epoch_tables`` the dynamic persistent kernel's tables come from."""
    E, n = P.shape
    pos_of = np.argsort(P, axis=1)
    k = pos_of[:, loc]
    rows = np.arange(E)[:, None]
    left = np.where(k > 0, P[rows, np.maximum(k - 1, 0)], -1)
    right = np.where(k + 1 < n, P[rows, np.minimum(k + 1, n - 1)], -1)
    li = np.broadcast_to(np.arange(len(loc)), k.shape)
    slots = np.stack([li, np.broadcast_to(loc, k.shape), left, right], axis=-1).astype(np.int32)
    return slots, k.astype(np.int32)


_QUAD_IDX: dict = {}
_QUAD_SRC: dict = {}


def quad_pad_image(M: torch.Tensor, db: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Lane-major image of the quad register layout of each (d, d) matrix in ``M`` (B, d, d), as
    ``quad_load_image`` in csrc/kernels/chain_blocked.hip reads it: lane l = i + 16c holds
    M[i + 16r, c + 4t] (r < 4, t < db / 4) at ((t >> 1) * 4 + r) * 128 + 2 l + (t & 1); zero outside d.
    Returns (B, 512 * ceil(db / 8)) float64 on M's device; on a HIP device with ``out`` given, written
    in place by one native launch (gadmm_pad_image_f64: the D-GADMM bench rebuilds it every solve)."""
    B, d = int(M.shape[0]), int(M.shape[1])
    qt = db // 4
    key = (d, db, M.device)
    idx = _QUAD_IDX.get(key)
    if idx is None:  # vectorised (a Python triple loop here cost ~45 ms on a process's first D-GADMM solve)
        n_el = 512 * ((qt + 1) // 2)
        src = np.full((n_el,), -1, dtype=np.int64)
        t, r, lane = np.meshgrid(np.arange(qt), np.arange(4), np.arange(64), indexing="ij")
        row, col = (lane & 15) + 16 * r, (lane >> 4) + 4 * t
        ok = (row < d) & (col < d)
        src[(((t >> 1) * 4 + r) * 128 + 2 * lane + (t & 1))[ok]] = (row * d + col)[ok]
        idx = (torch.from_numpy(np.maximum(src, 0)).to(M.device), torch.from_numpy(src >= 0).to(M.device))
        _QUAD_IDX[key] = idx
    gi, mask = idx
    if out is None and M.is_cuda and M.dtype == torch.float64:  # the native gather (torch.where's first
        out = torch.empty((B, int(gi.numel())), dtype=torch.float64, device=M.device)  # launch: ~90 ms)
    lib = native.require() if (out is not None and M.is_cuda) else None
    if lib is not None and hasattr(lib, "gadmm_pad_image_f64") and M.dtype == torch.float64 and M.is_contiguous():
        src = _QUAD_SRC.get(key)
        if src is None:
            src = torch.where(mask, gi, torch.full_like(gi, -1)).contiguous()
            _QUAD_SRC[key] = src
        fn = lib.gadmm_pad_image_f64
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                       ctypes.c_void_p, ctypes.c_void_p]
        native.check(fn(M.data_ptr(), d * d, src.data_ptr(), int(src.numel()), B, out.data_ptr(),
                        native.stream_handle()), "pad_image")
        return out
    flat = M.reshape(B, d * d).to(torch.float64)
    return torch.where(mask.unsqueeze(0), flat[:, gi], torch.zeros((), dtype=torch.float64, device=M.device)).contiguous()


def epoch_flush_table(P: np.ndarray, pos_of: Optional[np.ndarray] = None) -> np.ndarray:
    """(E, n, 2) int32: for epoch e >= 1 and chain position p, the OLD-chain neighbours (worker ids,
    -1 = none) of the worker that epoch e places at p, if that worker was a head of epoch e - 1's
    chain (a head's end-of-iteration dual is still pending at the re-chain and is flushed with them,
    dynamic_group_ADMM_closedForm.m:153-168); -1 everywhere for tails and for epoch 0. ``P``: (E, n)
    position -> worker; ``pos_of``: its inverse permutation per row (computed if None)."""
    P = np.asarray(P, dtype=np.int64)
    E, n = P.shape
    if pos_of is None:
        pos_of = np.argsort(P, axis=1)
    fl = np.full((E, n, 2), -1, dtype=np.int32)
    if E > 1:
        po = np.take_along_axis(pos_of[:-1], P[1:], axis=1)  # the new worker's old position
        was_head = (po % 2) == 0
        fl[1:, :, 0] = np.where(was_head & (po > 0), np.take_along_axis(P[:-1], np.maximum(po - 1, 0), axis=1), -1)
        fl[1:, :, 1] = np.where(was_head & (po < n - 1),
                                np.take_along_axis(P[:-1], np.minimum(po + 1, n - 1), axis=1), -1)
    return fl


class NativeChainEngine:
    def __init__(self, X_loc: torch.Tensor, y_loc: torch.Tensor, local_ids: Sequence[int], n_total: int,
                 model: str = "linear", rho: float = 1.0, obj0: float = 0.0, tol: float = 1e-4,
                 max_iter: int = 1000, lam: float = 0.0, step: float = 0.0, max_inner: int = 100,
                 inner_tol: float = 1e-4, comm=None, block: int = 16, stream: Optional[torch.cuda.Stream] = None,
                 precomputed=None, force_monitor: bool = False, obj_mode: str = "auto", local_solver: str = "gd",
                 chord: Optional[float] = None, residual: bool = False, xcd: int = 2):
        """``local_solver`` (logistic): "gd" = the reference's inexact inner GD (logReg_GD.m, step /
        max_inner / inner_tol), "newton" = exact local solves (group_ADMM_logistic.m semantics,
        csrc/kernels/chain_newton.hip; d, m <= 64). ``chord`` (newton): a worker reuses its last
        inverse Hessian while steps contract by at least this factor (0: refresh every step); None = the
        engine's default: 0.02 for the graph engine's phase kernels, 0.3 for the persistent kernel, whose
        crew refreshes the inverse in the background anyway (tools/newton_persist_tl.py --sweep: 424
        iterations at every setting, 9.31 / 8.00 / 7.87 ms at 0.02 / 0.1 / 0.3, profiles/r03_newton).
        ``obj_mode`` (graph / large-d phases): "exact" evaluates f_n = 1/2 th'A th - b'th + 1/2 y'y with a
        second GEMV by the Gram, "identity" uses A th = r - deg rho th from the solve itself (no second
        pass; at d > 256 that pass re-streams an 800 MB Gram per worker-phase), "auto" = identity at
        d > 256, exact otherwise (the verification path stays available as "exact").
        ``residual``: the kernels also emit the K4 primal residual (sum over chain edges of
        ||theta_n - theta_right||^2) per iteration, read back by ``primal_residual``. ``xcd`` (one GPU,
        persistent kernels): 0 default grid, 1 deal every working workgroup onto one XCD, 2 also
        publish with L2-resident plain stores once the kernel has verified that placement
        (PersistArgs::xcd; speed only, results are bit-identical)."""
        if not X_loc.is_cuda:
            raise ValueError("NativeChainEngine runs on a HIP device; use the torch algorithms on CPU")
        # the kernels read raw f64 pointers: anything else (e.g. float32 labels from torch.where) would be
        # reinterpreted bit for bit
        X_loc = X_loc.to(torch.float64)
        y_loc = y_loc.to(torch.float64)
        self.lib = native.require()
        self.device = X_loc.device
        self.model = model
        self.local_ids = [int(w) for w in local_ids]
        self.n_local = len(self.local_ids)
        self.n_total = int(n_total)
        self.d = int(X_loc.shape[2])
        self.m = int(X_loc.shape[1])
        self.comm = comm
        self.nranks = 1 if comm is None else comm.nranks
        # device-copy transport (parallel/ipc.py): replaces RCCL in the graph engine when present
        self.xport = getattr(comm, "xport", None) if comm is not None else None
        if local_solver not in ("gd", "newton"):
            raise ValueError("unknown local solver %r" % local_solver)
        if local_solver == "newton" and (model != "logistic" or self.d > 64 or self.m > 64):
            raise ValueError("native Newton local solves need the logistic model with d, m <= 64")
        self.local_solver = local_solver
        if force_monitor:
            # exercise the multi-rank stop path (partial-objective ring + RCCL all-reduce + monitor
            # kernel) with a 1-rank communicator: used by the single-GPU tests
            if comm is None:
                raise ValueError("force_monitor needs a communicator")
            self.nranks = 2
        self.block = int(block)
        self.ring = max(self.block, 1)
        # A dedicated (non-legacy) stream: hipGraph capture is not permitted on the null stream.
        self.stream = stream if stream is not None else torch.cuda.Stream(self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.rho, self.obj0, self.tol, self.max_iter = float(rho), float(obj0), float(tol), int(max_iter)
        dev, f64 = self.device, torch.float64
        d, nl = self.d, self.n_local

        with torch.cuda.stream(self.stream):
            self.theta = torch.zeros((self.n_total, d), dtype=f64, device=dev)
            self.mu = torch.zeros((nl, d), dtype=f64, device=dev)
            self.objw = torch.zeros((nl,), dtype=f64, device=dev)
            # read-back block, one device buffer so that a persistent solve's results come back in ONE
            # device-to-host copy: [ctl (8 x i32) | t0stamp | pad x 3 | trace (max_iter) | tstamp (max_iter)]
            mi = self.max_iter
            self._rb = torch.zeros((8 + 2 * mi,), dtype=f64, device=dev)
            self.ctl = self._rb[0:4].view(torch.int32)
            self.t0stamp = self._rb[4:5].view(torch.int64)
            self.trace = self._rb[8:8 + mi]
            self.trace.fill_(float("nan"))
            # multi-rank stop rule: per-worker objectives [ring][n_total] (gid-indexed, see gadmm_chain.h)
            self.part = torch.zeros((self.ring * self.n_total,), dtype=f64, device=dev)
            self.reduced = torch.zeros((self.ring * self.n_total,), dtype=f64, device=dev)
            self.lgid = torch.tensor(self.local_ids, dtype=torch.int32, device=dev)
            # real clock: s_memrealtime (100 MHz) of each iteration's decision (and t0stamp: the solve start)
            self.tstamp = self._rb[8 + mi:8 + 2 * mi].view(torch.int64)
            self.slots = torch.zeros((max(2 * nl, 2) * 4,), dtype=torch.int32, device=dev)
            self.inner_iters = torch.zeros((max(nl, 1),), dtype=torch.int32, device=dev)
            self.A = self.b = self.yy = self.Minv = None
            self.X = self.Y = None
            self.rbuf = None
            # Newton: per-worker inverse Hessian store (register image + valid flag + shift)
            self.hinv = torch.zeros((nl, 64 * 64 + 8), dtype=f64, device=dev) \
                if local_solver == "newton" and nl > 0 else None
            # the persistent Newton pipeline's refresh images (P | B | XP | XB per refresh slot, per worker)
            self.newton_img = torch.zeros((max(nl, 1) * int(native.require().gadmm_newton_rec_scratch_doubles()),),
                                          dtype=f64, device=dev) if local_solver == "newton" and nl > 0 else None
            self.chord = 0.02 if chord is None else float(chord)
            self.chord_persistent = 0.3 if chord is None else float(chord)
            self.xcd = int(xcd)
            # K4 primal residual: per (iteration, worker) contributions of the tails (owned rows only)
            self.rres = torch.zeros((self.max_iter * self.n_total,), dtype=f64, device=dev) if residual else None
            if d > 256:
                stride = int(native.require().gadmm_chain_big_rbuf_stride(d))
                self.rbuf = torch.zeros((max(nl, 1) * stride,), dtype=f64, device=dev)
            elif local_solver == "newton" and getenv("GADMM_NEWTON_TL") == "1":
                # instrumented Newton kernel: s_memrealtime stamps [n_local][50 steps][5] (tools/newton_stats.py)
                self.rbuf = torch.zeros((max(nl, 1) * 50 * 5,), dtype=torch.int64, device=dev)
            if model == "linear":
                if precomputed is not None:
                    self.A, self.b, self.yy = precomputed
                else:
                    self.A, self.b, self.yy = gram(X_loc, y_loc)
                self._build_inverses()
            elif model == "logistic":
                self.X = X_loc.contiguous()
                self.Y = y_loc.contiguous()
                self.nvar, self.deg_to_var = 1, (0, 0, 0)  # no cached inverses
            else:
                raise ValueError("unknown model %r" % model)

        args = native.PhaseArgs()
        args.d, args.n_local = d, nl
        args.nvar = self.nvar if model == "linear" else 1
        for i, v in enumerate(self.deg_to_var if model == "linear" else (0, 0, 0)):
            args.deg_to_var[i] = v
        args.model = native.MODEL_LINEAR if model == "linear" else native.MODEL_LOGISTIC
        args.Minv = native.ptr(self.hinv if self.hinv is not None else self._kernel_minv())
        args.A = native.ptr(self.A)
        args.b = native.ptr(self.b)
        args.yy = native.ptr(self.yy)
        args.mu = self.mu.data_ptr()
        args.theta = self.theta.data_ptr()
        args.rho = self.rho
        args.objw = self.objw.data_ptr()
        args.ctl = self.ctl.data_ptr()
        args.trace = self.trace.data_ptr()
        args.part = self.part.data_ptr()
        args.ring = self.ring
        args.max_iter = self.max_iter
        args.obj0, args.tol = self.obj0, self.tol
        args.X = native.ptr(self.X)
        args.Y = native.ptr(self.Y)
        args.m = self.m
        args.max_inner = int(max_inner)
        args.lam, args.step, args.inner_tol = float(lam), float(step), float(inner_tol)
        if local_solver == "newton":
            args.step = self.chord  # the Newton kernel's chord contraction threshold
        args.inner_iters = self.inner_iters.data_ptr()
        args.rbuf = native.ptr(self.rbuf)
        if obj_mode not in ("auto", "exact", "identity"):
            raise ValueError("unknown obj_mode %r" % obj_mode)
        args.obj_mode = 0 if (obj_mode == "exact" or (obj_mode == "auto" and d <= 256)) else 1
        self.obj_mode_name = "exact" if args.obj_mode == 0 else "identity"
        args.solver = 1 if local_solver == "newton" else 0
        args.n_total = self.n_total
        args.lgid = self.lgid.data_ptr()
        args.tstamp = self.tstamp.data_ptr()
        args.rres = native.ptr(self.rres)
        desc = native.EngineDesc()
        desc.base = args
        desc.d_slots = self.slots.data_ptr()
        desc.reduced = self.reduced.data_ptr()
        desc.comm = comm.handle if comm is not None else None
        desc.stream = self.stream.cuda_stream
        desc.nranks = self.nranks
        desc.xport = self.xport
        self._desc = desc
        self.handle = self.lib.gadmm_chain_engine_create(ctypes.byref(desc))
        if not self.handle:
            native.check(-1, "chain_engine_create")
        self.plan: Optional[RankPlan] = None
        self.path: Optional[List[int]] = None
        self._pbuf = None

    # ---------------------------------------------------------------------------------------------
    def _build_inverses(self, in_place: bool = False, check: bool = True):
        self._minv_version = getattr(self, "_minv_version", 0) + 1  # the blocked D-GADMM pad follows it
        rho = self.rho
        if self.n_total == 1:
            shifts, self.deg_to_var = [0.0], (0, 0, 0)
        elif self.n_total == 2:  # both workers are chain ends in every chain: degree 1 only
            shifts, self.deg_to_var = [rho], (0, 0, 0)
        else:
            shifts, self.deg_to_var = [rho, 2.0 * rho], (0, 0, 1)
        self.nvar = len(shifts)
        key = (tuple(shifts), self.A.shape[0])
        if getattr(self, "_shift_key", None) != key or not in_place:
            self._refresh_fast = None  # its bound arguments name the shifts / inverse buffers
        if getattr(self, "_shift_key", None) != key:  # (N, V) shifts + status word, built once per rho
            self._shift_key = key
            self._shifts = torch.tensor(shifts, dtype=torch.float64, device=self.device).unsqueeze(0).expand(
                self.A.shape[0], -1).contiguous()
            self._inv_status = torch.zeros((1,), dtype=torch.int32, device=self.device)
        st = None if check else self._inv_status  # the cached word only where nobody reads it back
        if in_place and self.Minv is not None:
            spd_inverse(self.A, self._shifts, out=self.Minv, check_status=check, status=st)
        else:
            self.Minv = spd_inverse(self.A, self._shifts, check_status=check, status=st)
        if self.d > 256:
            # the large-d phases (chain_big.hip) stream the block-packed lower triangles: half the bytes
            self.Mpk = sym_pack(self.Minv, out=self.Mpk if in_place and getattr(self, "Mpk", None) is not None
                                else None)

    def _kernel_minv(self):
        """The inverses as the phase kernels read them: block-packed lower triangles at d > 256."""
        return getattr(self, "Mpk", None) if self.d > 256 else self.Minv

    def refresh(self, X_loc: torch.Tensor, y_loc: torch.Tensor):
        """Recompute the loop-invariant set-up (Gram + cached inverses) from the raw shards, in place
        (device pointers, hence captured graphs, stay valid). No host synchronisation.
        Repeated refreshes of the same shards at d <= 128 (every bench step) take a prebound path: the
        Gram and inverse launches go straight to the native library on the engine stream with their
        arguments built once (the general path's torch stream context, workspace allocation and
        argument checks were ~20 us of host time per solve, on the critical path of a 1 ms D-GADMM
        solve). Same kernels, same arguments: bit-identical."""
        fast = getattr(self, "_refresh_fast", None)
        if fast is not None and fast[0] is X_loc and fast[1] is y_loc:
            lib, g_args, i_args = fast[2], fast[3], fast[4]
            native.check(lib.gadmm_gram_f64(*g_args), "gram_f64")
            native.check(lib.gadmm_spd_inverse_small_f64(*i_args), "spd_inverse_small_f64")
            self._minv_version = getattr(self, "_minv_version", 0) + 1
            pf = getattr(self, "_pad_fast", None)
            if pf is not None and pf[0] is self.Minv and pf[1] is getattr(self, "_minv_pad", None):
                # the blocked D-GADMM inverse image follows at once, queued behind the inverses: built
                # in run_persistent it sat between the epoch-table copy and the launch (profiles/r06_dgadmm)
                native.check(lib.gadmm_pad_image_f64(*pf[2]), "pad_image")
                self._minv_pad_version = self._minv_version
            return
        if (self.model == "linear" and X_loc.is_cuda and self.d <= 128 and X_loc.dtype == torch.float64
                and y_loc.dtype == torch.float64 and X_loc.is_contiguous() and y_loc.is_contiguous()
                and tuple(X_loc.shape) == (self.n_local, self.m, self.d) and self.Minv is not None
                and getattr(self, "_shifts", None) is not None and getattr(self, "_inv_status", None) is not None):
            lib = self.lib
            N, m, d = int(X_loc.shape[0]), int(X_loc.shape[1]), int(X_loc.shape[2])
            ks = int(lib.gadmm_gram_pick_ksplit(N, m, d))
            ws_n = int(lib.gadmm_gram_workspace(N, m, d, ks))
            self._refresh_ws = torch.empty((max(ws_n, 1),), dtype=torch.float64, device=self.device) \
                if ws_n > 0 else None
            st = self.stream.cuda_stream
            g_args = (X_loc.data_ptr(), y_loc.data_ptr(), N, m, d, ks, self.A.data_ptr(), self.b.data_ptr(),
                      self.yy.data_ptr(), self._refresh_ws.data_ptr() if self._refresh_ws is not None else None, st)
            i_args = (self.A.data_ptr(), self._shifts.data_ptr(), N, d, int(self._shifts.shape[1]),
                      self.Minv.data_ptr(), self._inv_status.data_ptr(), st)
            self._refresh_fast = (X_loc, y_loc, lib, g_args, i_args)
            return self.refresh(X_loc, y_loc)
        with torch.cuda.stream(self.stream):
            if self.model == "linear":
                gram(X_loc, y_loc, out=(self.A, self.b, self.yy))
                self._build_inverses(in_place=True, check=False)
            else:
                self.X.copy_(X_loc)
                self.Y.copy_(y_loc)

    def set_rho(self, rho: float):
        """Change rho (re-inverts; the Gram is kept)."""
        self.rho = float(rho)
        if self.model == "linear":
            with torch.cuda.stream(self.stream):
                self._build_inverses()
            self._desc.base.Minv = self._kernel_minv().data_ptr()
        self._desc.base.rho = self.rho
        self._recreate()

    def _recreate(self):
        self.lib.gadmm_chain_engine_destroy(self.handle)
        self.handle = self.lib.gadmm_chain_engine_create(ctypes.byref(self._desc))
        if self.plan is not None:
            self._install(self.plan)
            self._plan_dirty = False

    def set_targets(self, obj0: float, tol: float, max_iter: Optional[int] = None):
        self.obj0, self.tol = float(obj0), float(tol)
        if max_iter is not None and max_iter != self.max_iter:
            raise ValueError("max_iter is fixed at construction (trace buffer size)")
        native.check(self.lib.gadmm_chain_engine_set_scalars(self.handle, self.rho, self.obj0, self.tol,
                                                             self.max_iter), "set_scalars")
        self._desc.base.obj0, self._desc.base.tol = self.obj0, self.tol

    # ---------------------------------------------------------------------------------------------
    def set_path(self, path: Sequence[int], placement: Placement, rank: int):
        """Install the chain ``path`` (position -> global worker id) for this rank."""
        # validated plans are memoised per (chain, rank, placement): a D-GADMM solve installs the same
        # initial and final chains on every repeat, and building a plan in Python costs ~50 us
        pl = path.tolist() if isinstance(path, np.ndarray) else [int(w) for w in path]
        ok = getattr(self, "_owner_memo", None)  # the placement's owner tuple, memoised per object
        if ok is None or ok[0] is not placement:
            ok = (placement, tuple(int(o) for o in placement.owner))
            self._owner_memo = ok
        key = (tuple(pl), int(rank), ok[1])
        memo = self.__dict__.setdefault("_plan_memo", {})
        plan = memo.get(key)
        if plan is None:
            plan = chain_plan(pl, placement, rank)
            lidx = {w: i for i, w in enumerate(self.local_ids)}
            for s in plan.head + plan.tail:
                if self.local_ids[s.li] != s.gid or lidx[s.gid] != s.li:
                    raise ValueError("placement/local_ids mismatch")
            if len(memo) > 4096:
                memo.clear()
            memo[key] = plan
        # installed into the native engine lazily (_sync_plan): the persistent kernels take their slots
        # from self.plan, and a D-GADMM solve re-installs its final chain after every launch
        if plan is not getattr(self, "plan", None):
            self._plan_dirty = True
        self.plan = plan
        self.path = pl
        self.rank = rank
        self._placement_owner = list(ok[1])

    def _sync_plan(self):
        """Install self.plan into the native (graph / eager) engine if set_path changed it."""
        if getattr(self, "_plan_dirty", False) and self.plan is not None:
            self._install(self.plan)
            self._plan_dirty = False

    def _install(self, plan: RankPlan):
        def slots(lst):
            arr = (native.PhaseSlot * max(len(lst), 1))()
            for i, s in enumerate(lst):
                arr[i].li, arr[i].gid, arr[i].left, arr[i].right = s.li, s.gid, s.left, s.right
            return arr

        def ops(lst):
            arr = (native.XchgOp * max(len(lst), 1))()
            for i, (peer, row, snd) in enumerate(lst):
                arr[i].peer, arr[i].row, arr[i].is_send, arr[i].count = peer, row, snd, 0
            return arr

        if len(plan.head) + len(plan.tail) > 2 * max(self.n_local, 1):
            raise ValueError("plan larger than slot buffer")
        rc = self.lib.gadmm_chain_engine_set_plan(self.handle, len(plan.head), slots(plan.head), len(plan.tail),
                                                  slots(plan.tail), len(plan.xchg_head), ops(plan.xchg_head),
                                                  len(plan.xchg_tail), ops(plan.xchg_tail))
        native.check(rc, "set_plan")

    def reset(self, start_iter: int = 1, pending: int = 0, zero_state: bool = True):
        self._tr_valid = False
        if self.xport:  # new solve: the transport's tags of the previous one stop matching (every rank)
            native.check(self.lib.gadmm_ipc_new_epoch(self.xport, self.stream.cuda_stream), "ipc_new_epoch")
        if not zero_state:
            native.check(self.lib.gadmm_write_stamp(self.t0stamp.data_ptr(), self.stream.cuda_stream), "write_stamp")
        if self.hinv is not None and zero_state:  # a new solve starts from fresh Hessians
            with torch.cuda.stream(self.stream):
                self.hinv[:, 64 * 64].zero_()
        if self.rres is not None and zero_state:  # a row's non-tail entries stay 0
            with torch.cuda.stream(self.stream):
                self.rres.zero_()
        if zero_state:  # theta = mu = part = 0, trace = NaN, the control block and the clock start: one launch
            native.check(self.lib.gadmm_chain_reset_state_stamp(
                self.ctl.data_ptr(), int(start_iter), int(pending), self.theta.data_ptr(), self.theta.numel(),
                self.mu.data_ptr(), self.mu.numel(), self.trace.data_ptr(), self.trace.numel(),
                self.part.data_ptr(), self.part.numel(), self.t0stamp.data_ptr(), self.stream.cuda_stream),
                "reset_state")
        else:
            native.check(self.lib.gadmm_chain_engine_reset(self.handle, int(start_iter), int(pending)), "reset")

    def exchange(self, which: str = "tail"):
        """Eager neighbour exchange with the current plan ('head' or 'tail' messages)."""
        self._sync_plan()
        native.check(self.lib.gadmm_chain_engine_exchange(self.handle, 0 if which == "head" else 1), "exchange")

    def flush_duals(self):
        """Apply pending head duals with the current chain (before re-chain / checkpoint)."""
        self._sync_plan()
        native.check(self.lib.gadmm_chain_engine_flush(self.handle), "flush")

    def run(self, stop_iter: int = 0, use_graph: bool = True, block: Optional[int] = None) -> EngineRun:
        self._tr_valid = False
        st = native.RunStats()
        blk = self.block if block is None else int(block)
        if blk > self.ring and self.nranks > 1:
            raise ValueError("block must be <= ring for multi-rank runs")
        self._sync_plan()
        # the watchdog of the host waits: an RCCL data plane has no deadline of its own (the engine
        # aborts the communicator when it passes; native.RcclDead / NativeTimeout reach the caller)
        tmo = float(getattr(self.comm, "timeout_s", 0.0) or 0.0) if getattr(self.comm, "backend", "") == "rccl" else 0.0
        native.check(self.lib.gadmm_chain_engine_set_timeout(self.handle, tmo), "chain_engine_set_timeout")
        rc = self.lib.gadmm_chain_engine_run(self.handle, blk, int(stop_iter), 1 if use_graph else 0,
                                             ctypes.byref(st))
        native.check(rc, "chain_engine_run")
        return EngineRun(st.iters, st.done, st.iterations_launched, st.replays, st.wall_ms, st.p2p_bytes,
                         st.p2p_msgs, st.monitor_bytes, st.wire_bytes)

    # ---------------------------------------------------------------------------------------------
    # Persistent single-launch solve (csrc/kernels/chain_persistent.hip)
    def resident_capacity(self, dynamic: bool = False, sys_scope: bool = False) -> int:
        """Workgroups of the per-worker persistent kernel this device can keep resident at once
        (occupancy x CUs, ``GADMM_CU_BUDGET`` shrinks the CU count): a persistent launch needs all of
        them together, so eligibility is decided here, up front, not by a spin deadline."""
        # memoised per (mode, the env switches the launcher reads): a D-GADMM solve asks on every call
        key = (bool(dynamic), bool(sys_scope), getenv("GADMM_CU_BUDGET"), getenv("GADMM_PERSIST_LDS"))
        memo = self.__dict__.setdefault("_cap_memo", {})
        if key not in memo:
            pa = native.PersistArgs()
            pa.d, pa.n, pa.nvar, pa.obj_mode = self.d, self.n_total, self.nvar, self._obj_mode(dynamic)
            pa.n_epochs = 1 if dynamic else 0
            pa.sys_scope = 1 if sys_scope else 0
            memo[key] = int(self.lib.gadmm_chain_persistent_capacity(ctypes.byref(pa)))
        return memo[key]

    def _logi_args(self) -> native.LogiArgs:
        g = native.LogiArgs()
        b = self._desc.base
        g.X, g.Y, g.m, g.max_inner = native.ptr(self.X), native.ptr(self.Y), self.m, int(b.max_inner)
        g.lam, g.step, g.inner_tol = float(b.lam), float(b.step), float(b.inner_tol)
        if self.local_solver == "newton":
            g.step = self.chord_persistent  # the persistent Newton kernel's chord contraction threshold
        g.inner_iters = self.inner_iters.data_ptr()
        g.scratch = self.newton_img.data_ptr() if self.newton_img is not None else None
        return g

    def persistent_eligible(self, fabric=None) -> bool:
        if self.plan is None or self.path is None:
            return False
        if self.nranks != 1 and fabric is None:
            return False
        if self.model == "logistic":
            # logistic in one launch: inner GD (chain_persistent_logistic.hip, one wave per worker) or
            # exact Newton (chain_persistent_newton.hip: a solver wave + a 4-wave crew that rebuilds the
            # inverse Hessian off the critical path; d, m <= 52; GADMM_NEWTON_PERSISTENT=0: graph engine)
            if max(self.d, self.m) > 64:
                return False
            pa = native.PersistArgs()
            pa.d, pa.n, pa.sys_scope = self.d, self.n_total, 1 if fabric is not None else 0
            g = self._logi_args()
            if self.local_solver == "newton":
                if getenv("GADMM_NEWTON_PERSISTENT", "1") == "0":
                    return False
                cap = int(self.lib.gadmm_chain_persistent_newton_capacity(ctypes.byref(pa), ctypes.byref(g)))
            else:
                cap = int(self.lib.gadmm_chain_persistent_logistic_capacity(ctypes.byref(pa), ctypes.byref(g)))
            return self.n_local + 1 <= cap
        if self.model != "linear":
            return False
        if self._lds_need(False, self._obj_mode()) <= 0:
            return False
        return self.n_local + 1 <= self.resident_capacity(sys_scope=fabric is not None)

    def _lds_need(self, dynamic: bool, obj_mode: int) -> int:
        """LDS bytes of the per-worker persistent kernel (gadmm_chain_persistent_lds[_dyn]; <= 0: does
        not fit), memoised: a pure function of (d, nvar, mode), asked several times per solve."""
        memo = self.__dict__.setdefault("_lds_memo", {})
        key = (bool(dynamic), int(obj_mode))
        v = memo.get(key)
        if v is None:
            v = int(self.lib.gadmm_chain_persistent_lds_dyn(self.d, obj_mode, self.nvar) if dynamic
                    else self.lib.gadmm_chain_persistent_lds(self.d, obj_mode))
            memo[key] = v
        return v

    def _obj_mode(self, dynamic: bool = False) -> int:
        # exact objective (second GEMV with the Gram in LDS) whenever both matrices fit in LDS
        return 0 if self._lds_need(dynamic, 0) > 0 else 1

    # coherence (iterations per epoch) from which the blocked kernel's dynamic mode is the default:
    # measured per solve (profiles/r03_dgadmm_rechain) 1.01 vs 1.47 ms at coherence 10, 0.96 vs 1.12 ms
    # at 3, but 1.38 vs 1.16 ms at 1 (every iteration re-chains)
    BLOCKED_DYN_MIN_COHERENCE = 3

    def dynamic_uses_blocked(self, fabric=None, coherence=None) -> bool:
        """Whether a one-launch D-GADMM run takes the blocked kernel's dynamic mode (one GPU, 12-wave
        layout) rather than the per-worker kernel: GADMM_BLOCKED_DYN=1 / 0 forces it on / off; unset,
        it is on when the schedule re-chains every ``BLOCKED_DYN_MIN_COHERENCE`` or more iterations
        (``coherence``; None: off). Both run epoch chunks (hard stop + continuation)."""
        plan = self.blocked_plan(fabric) if self.model == "linear" else None
        if plan is None or plan[3] != 1 or self.n_local != self.n_total:
            return False
        env = getenv("GADMM_BLOCKED_DYN", "")
        if env in ("0", "1"):
            return env == "1"
        return coherence is not None and float(coherence) >= self.BLOCKED_DYN_MIN_COHERENCE

    def dynamic_eligible(self, fabric=None) -> bool:
        """One-launch D-GADMM (per-epoch chains in device tables): linear, every degree's inverse
        resident; several ranks need an xGMI fabric whose theta tables hold a ring of iteration slots."""
        if self.model != "linear":
            return False
        if self.nranks != 1 and (fabric is None or getattr(fabric, "table_slots", 1) < 2):
            return False
        if self.nranks == 1 and self.n_local != self.n_total:
            return False
        if self._lds_need(True, self._obj_mode(True)) <= 0:
            return False
        return self.n_local + 1 <= self.resident_capacity(dynamic=True, sys_scope=fabric is not None)

    def blocked_plan(self, fabric=None, timeline: bool = False):
        """(k, L, W, pw) of the temporally blocked kernel for this engine, or None (multi-GPU, d > 64,
        GADMM_BLOCKED=0). pw = positions per wave: 1 = the 12-wave kernel (default, also the only
        instrumented one, so ``timeline`` selects it), 2 = the paired 8-wave kernel (GADMM_BLOCK_PW=2)."""
        if fabric is not None or self.nranks > 1 or self.d > 64 or getenv("GADMM_BLOCKED", "1") == "0":
            return None
        # memoised per (timeline, the env switches the planner reads)
        key = (bool(timeline), getenv("GADMM_BLOCK_K"), getenv("GADMM_BLOCK_L"),
               getenv("GADMM_BLOCK_PW"), getenv("GADMM_CU_BUDGET"))
        memo = self.__dict__.setdefault("_plan2_memo", {})
        if key not in memo:
            kk, ll, pp = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
            want = int(getenv("GADMM_BLOCK_K", "0"))
            W = int(self.lib.gadmm_chain_blocked_plan2(self.n_total, self.d, want, 1 if timeline else 0,
                                                       ctypes.byref(kk), ctypes.byref(ll), ctypes.byref(pp)))
            memo[key] = (kk.value, ll.value, W, pp.value) if W > 0 else None
        return memo[key]

    def run_persistent(self, lag: int = 4, timeout_s: float = 20.0, start_iter: int = 1,
                       pending_in: int = 0, fabric=None, timeline_iters: int = 0,
                       epochs: Optional[Sequence] = None, hard_stop: int = 0, cont: bool = False,
                       fetch_trace: bool = False, blocked_dyn: Optional[bool] = None,
                       on_enqueued=None) -> EngineRun:
        """Whole solve in one launch per GPU. State must be reset (``reset()``) or resumed by the
        caller. ``fabric``: an ``XgmiFabric`` for the multi-GPU device-initiated transport.
        ``timeline_iters > 0`` records s_memrealtime stamps (10 ns) of the first iterations into
        ``self.last_timeline``: (workgroup, iteration, [start, ready, published, end, after the
        barrier, after the solve GEMV, -, -]); the last
        workgroup row is the monitor (column 0 = decision posted).
        ``epochs``: D-GADMM in one launch, a list of ``(first_iteration, path)`` or a pair of arrays
        ``(first_iterations (E,), paths (E, n))`` (the first epoch starts at ``start_iter``); every worker switches neighbours / role at each epoch start and flushes its
        pending head dual with the old chain first. With a ``fabric`` (several GPUs) each worker also
        pushes its theta to the ranks of its current and next-epoch neighbours (the fabric's theta
        tables must hold ``table_slots >= lag + 4`` iteration slots).
        Epoch chunks (D-GADMM, per-worker kernel): ``hard_stop > 0`` runs no iteration past it (the
        monitor rank's ``done`` is then 5 unless it decided a stop; the table should include the epoch
        starting at ``hard_stop + 1``, whose neighbours receive theta^hard_stop); ``cont=True`` continues
        the previous chunk from ``start_iter = hard_stop + 1`` with the same tag salt, epoch 0 being the
        previous chunk's last epoch (its heads' pending duals are flushed with that chain).
        ``fetch_trace``: the objective trace and clock come back behind the same stream sync (for a
        caller that reads ``traces()`` next; a benchmark loop that does not leaves it off).
        ``blocked_dyn``: D-GADMM on the blocked kernel's dynamic mode (None: ``dynamic_uses_blocked``).
        ``on_enqueued``: a host callback run after the launch and its read-back copy are queued and
        before the stream is synchronised -- host work of the caller that does not need the outcome
        (e.g. D-GADMM's per-epoch cost arrays) overlaps the kernel instead of following it."""
        _timing.host_stamp("rp:start")
        if epochs is not None:
            if not self.dynamic_eligible(fabric):
                raise RuntimeError("dynamic persistent kernel not eligible for this engine/config")
        elif not self.persistent_eligible(fabric):
            raise RuntimeError("persistent kernel not eligible for this engine/config")
        plan = self.blocked_plan(fabric, timeline=timeline_iters > 0) if self.model == "linear" else None
        if blocked_dyn is None:
            blocked_dyn = self.dynamic_uses_blocked(fabric)
        if epochs is not None and (not blocked_dyn or timeline_iters > 0):
            # D-GADMM on the per-worker kernel unless the blocked kernel's dynamic mode is selected
            # (dynamic_uses_blocked); both run epoch chunks (hard stop + continuation)
            plan = None
        if plan is not None:
            lag = max(lag, 8)  # the objective takes one more hop (worker -> objective wave -> monitor)
        ring = lag + 4
        dev = self.device
        # this rank's slots in chain order, their positions and the buffer key: memoised per plan
        pk = (id(self.plan), tuple(self.path))
        memo = getattr(self, "_slot_memo", None)
        if memo is None or memo[0] != pk:
            pos_of = {g: i for i, g in enumerate(self.path)}
            sl = sorted(self.plan.head + self.plan.tail, key=lambda s: pos_of[s.gid])
            memo = (pk, sl, [pos_of[s.gid] for s in sl], tuple((s.li, s.gid, s.left, s.right) for s in sl), self.plan)
            self._slot_memo = memo
        _, slots, pos, slot_key, _ = memo
        key = (ring, slot_key, id(fabric), epochs is not None)
        if getattr(self, "_pbuf", None) is None or self._pbuf[0] != key:
            with torch.cuda.stream(self.stream):
                slot_t = torch.tensor([[s.li, s.gid, s.left, s.right] for s in slots], dtype=torch.int32,
                                      device=dev).reshape(-1)
                pos_t = torch.tensor(pos, dtype=torch.int32, device=dev)
                if fabric is None:
                    # D-GADMM (epochs): one theta slot per ring iteration (see chain_persistent.hip)
                    thg = torch.zeros(((ring if epochs is not None else 1) * self.n_total * self.d * 4,),
                                      dtype=torch.int32, device=dev)
                    objg = torch.zeros((ring * self.n_total * 4,), dtype=torch.int32, device=dev)
                    decg = torch.zeros((ring,), dtype=torch.int64, device=dev)
                    ptrs = (thg.data_ptr(), objg.data_ptr(), decg.data_ptr())
                    push = None
                    dec_push = torch.tensor([decg.data_ptr()], dtype=torch.int64, device=dev)
                    keep = (thg, objg, decg)
                elif epochs is not None:
                    # D-GADMM across GPUs: push targets change per epoch (ep_push masks below)
                    if getattr(fabric, "table_slots", 1) < ring:
                        raise RuntimeError("fabric theta tables hold %d slots, D-GADMM needs %d"
                                           % (getattr(fabric, "table_slots", 1), ring))
                    push = None
                else:
                    owner = self._placement_owner
                    pl = []
                    for s in slots:
                        peers = sorted({int(owner[u]) for u in (s.left, s.right) if u >= 0} - {self.rank})
                        ps = [fabric.thg_peer[r] for r in peers] + [0, 0]
                        pl += ps[:2]
                    push = torch.tensor(pl, dtype=torch.int64, device=dev)
                if fabric is not None:
                    ptrs = (fabric.thg.ptr.value, fabric.objg_mon, fabric.decg.ptr.value)
                    dec_push = torch.tensor(fabric.dec_all if fabric.dec_all else [0], dtype=torch.int64,
                                            device=dev)
                    keep = (torch.tensor(fabric.table_ptrs(), dtype=torch.int64, device=dev),) \
                        if epochs is not None else ()
            self._pbuf = (key, slot_t, pos_t, ptrs, push, dec_push, keep, [0])
        _, slot_t, pos_t, ptrs, push, dec_push, keep, epoch_box = self._pbuf
        if cont:  # same salt: the tables still hold theta^{start_iter - 1} of the previous chunk
            epoch = self._salt
            native.check(self.lib.gadmm_chain_engine_reset(self.handle, int(start_iter), int(pending_in)), "reset")
        elif fabric is not None:
            epoch = fabric.next_epoch()
        else:
            epoch_box[0] = epoch_box[0] % 4095 + 1
            epoch = epoch_box[0]
        self._salt = epoch
        if fabric is None and getattr(self, "_xchk", None) is None:  # XCD packing (one GPU): PersistArgs::xcd
            # zeroed on the engine stream, ordered before the kernel: a fill on torch's current stream
            # could land while the blocks post their placement granules (they then spin to the deadline)
            with torch.cuda.stream(self.stream):
                self._xchk = torch.zeros((256 * 4,), dtype=torch.int32, device=dev)
        # the launch-invariant fields, set once per (buffers, targets, layout) and copied per launch (a
        # D-GADMM solve launches every ~1 ms: ~40 ctypes field stores were ~3 us of its host path). The
        # buffers are held by the key itself, compared by identity, so a freed one cannot alias a new one
        objs = (self._pbuf, self.Minv, self.A, self.b, self.yy, self.theta, self.mu, self.trace, self.ctl,
                self.tstamp, self.rres, fabric, getattr(self, "_xchk", None))
        nums = (int(lag), ring, self.rho, self.obj0, self.tol, float(timeout_s), epochs is not None, self.rank,
                self.nranks, int(self.xcd), self.nvar, tuple(self.deg_to_var), self.max_iter, len(slots))
        tmpl = self.__dict__.get("_pa_tmpl")
        if tmpl is None or tmpl[1] != nums or any(x is not y for x, y in zip(tmpl[0], objs)):
            pt = native.PersistArgs()
            pt.d, pt.n, pt.n_local, pt.max_iter = self.d, self.n_total, len(slots), self.max_iter
            pt.lag, pt.ring, pt.nvar, pt.obj_mode = int(lag), ring, self.nvar, self._obj_mode(epochs is not None)
            for i, v in enumerate(self.deg_to_var):
                pt.deg_to_var[i] = v
            pt.has_monitor = 1 if (fabric is None or self.rank == 0) else 0
            pt.nranks = 1 if fabric is None else self.nranks
            pt.sys_scope = 0 if fabric is None else 1
            pt.rho, pt.obj0, pt.tol = self.rho, self.obj0, self.tol
            pt.timeout_ticks = int(timeout_s * 1e8)
            pt.slots, pt.pos = slot_t.data_ptr(), pos_t.data_ptr()
            pt.Minv, pt.A, pt.b, pt.yy = native.ptr(self.Minv), native.ptr(self.A), native.ptr(self.b), native.ptr(self.yy)
            pt.theta, pt.mu = self.theta.data_ptr(), self.mu.data_ptr()
            pt.thg, pt.objg, pt.decg = ptrs
            pt.push = push.data_ptr() if push is not None else None
            pt.dec_push = dec_push.data_ptr()
            pt.trace, pt.ctl = self.trace.data_ptr(), self.ctl.data_ptr()
            pt.tstamp = self.tstamp.data_ptr()
            pt.rres = native.ptr(self.rres)
            if fabric is None:
                pt.xchk, pt.xcd = self._xchk.data_ptr(), int(self.xcd)
            tmpl = (objs, nums, pt)
            self._pa_tmpl = tmpl
        pa = native.PersistArgs.from_buffer_copy(tmpl[2])
        pa.start_iter, pa.pending_in, pa.epoch = int(start_iter), int(pending_in), int(epoch)
        pa.hard_stop, pa.cont = int(hard_stop), 1 if cont else 0
        _timing.host_stamp("rp:args")
        fused = epochs is not None and plan is not None and fabric is None and isinstance(epochs, tuple) \
            and len(epochs) == 2 and isinstance(epochs[1], np.ndarray) and isinstance(epochs[0], np.ndarray) \
            and epochs[0].dtype == np.int64 and epochs[1].dtype == np.int64 and epochs[1].flags.c_contiguous \
            and epochs[0].flags.c_contiguous
        if fused:
            # blocked kernel on one GPU: checks, tables, staging and the H2D copy in one native call
            # (gadmm_epoch_stage_blocked), the layout of the general path below with no push masks
            starts, P = epochs
            E, n = P.shape
            total = E + 7 * E * n
            stage = getattr(self, "_ep_stage", None)
            if stage is None or stage[0].numel() < total:
                cap = max(total, 4096)
                h_t = torch.empty((cap,), dtype=torch.int32, pin_memory=True)
                d_t = torch.empty((cap,), dtype=torch.int32, device=dev)
                stage = (h_t, d_t, h_t.numpy(), h_t.data_ptr(), d_t.data_ptr())
                self._ep_stage = stage
            if len(starts) != E:
                raise ValueError("epochs: one chain per start")
            got = int(self.lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P.ctypes.data, E, n, int(start_iter),
                                                         1 if cont else 0, stage[3], stage[0].numel(), stage[4],
                                                         self.stream.cuda_stream))
            if got < 0:
                raise ValueError(self.lib.gadmm_last_error().decode())
            dptr = stage[4]
            pa.n_epochs = E
            pa.epoch_start, pa.ep_slots = dptr, dptr + 4 * E
            pa.ep_pos, pa.ep_flush = dptr + 4 * (E + 4 * E * n), dptr + 4 * (E + 5 * E * n)
        elif epochs is not None:
            if isinstance(epochs, tuple) and len(epochs) == 2 and isinstance(epochs[1], np.ndarray):
                starts = np.asarray(epochs[0], dtype=np.int64)                      # (starts, paths) arrays
                P = np.asarray(epochs[1], dtype=np.int64)
            else:
                starts = np.asarray([int(e[0]) for e in epochs], dtype=np.int64)
                P = np.asarray([list(e[1]) for e in epochs], dtype=np.int64)       # (E, n) position -> worker
            if (starts[0] > int(start_iter) if cont else starts[0] != int(start_iter)) or np.any(starts[1:] <= starts[:-1]):
                raise ValueError("epochs must start at start_iter (continuations: at or before it) and increase")
            E, n = P.shape
            if E != len(starts):
                raise ValueError("epochs: one chain per start")
            loc = np.asarray([int(w) for w in self.local_ids], dtype=np.int64)
            if plan is not None:
                # blocked kernel (one GPU, every worker local: li == worker id): slots in chain-POSITION
                # order per epoch (li, gid, left, right), worker -> position, and the flush pairs
                # (PersistArgs::ep_flush) -- native C++ builder (csrc/runtime/topology.cpp; the numpy
                # equivalent is epoch_flush_table + fancy indexing)
                P = np.ascontiguousarray(P)
                es = np.empty((E * n * 4,), dtype=np.int32)
                pp = np.empty((E * n,), dtype=np.int32)
                fl = np.empty((E * n * 2,), dtype=np.int32)
                native.check(self.lib.gadmm_epoch_tables_blocked(P.ctypes.data, E, n, es.ctypes.data, pp.ctypes.data,
                                                                 fl.ctypes.data), "epoch_tables_blocked")
            else:
                # per-worker kernel: the slot / position of every LOCAL worker per epoch (native C++
                # builder, csrc/runtime/topology.cpp; the numpy equivalent is epoch_tables_numpy)
                P = np.ascontiguousarray(P)
                es = np.empty((E * len(loc) * 4,), dtype=np.int32)
                pp = np.empty((E * len(loc),), dtype=np.int32)
                native.check(self.lib.gadmm_epoch_tables(P.ctypes.data, E, n, loc.ctypes.data, len(loc),
                                                         es.ctypes.data, pp.ctypes.data), "epoch_tables")
            # the three epoch tables go up in ONE async copy from a reused pinned staging buffer (three
            # pageable copies cost a blocking round trip each); the stream is synchronised after the
            # kernel, so the staging buffer is free again by the next solve
            if fabric is not None:
                # ranks each local worker pushes theta to in each epoch: its neighbours' owners
                owner = np.asarray(self._placement_owner, dtype=np.int64)
                sl4 = es.reshape(E, len(loc), 4)
                mask = np.zeros((E, len(loc)), dtype=np.int64)
                for col in (2, 3):
                    nb = sl4[:, :, col].astype(np.int64)
                    ow = np.where(nb >= 0, owner[np.maximum(nb, 0)], self.rank)
                    mask |= np.where(ow != self.rank, np.left_shift(1, ow), 0)
                pm = mask.astype(np.int32).reshape(-1)
            else:
                pm = np.zeros((0,), dtype=np.int32)
            if plan is None:
                fl = np.zeros((0,), dtype=np.int32)
            ns, nes = len(starts), es.size
            total = ns + nes + pp.size + pm.size + fl.size
            stage = getattr(self, "_ep_stage", None)
            if stage is None or stage[0].numel() < total:
                cap = max(total, 4096)
                h_t = torch.empty((cap,), dtype=torch.int32, pin_memory=True)
                d_t = torch.empty((cap,), dtype=torch.int32, device=dev)
                stage = (h_t, d_t, h_t.numpy(), h_t.data_ptr(), d_t.data_ptr())
                self._ep_stage = stage
            host, hptr, dptr = stage[2], stage[3], stage[4]
            o_es, o_pp, o_pm, o_fl = ns, ns + nes, ns + nes + pp.size, total - fl.size
            host[:ns] = starts
            host[o_es:o_pp] = es
            host[o_pp:o_pm] = pp
            host[o_pm:o_fl] = pm
            host[o_fl:total] = fl
            native.check(self.lib.gadmm_memcpy_h2d_async(dptr, hptr, total * 4, self.stream.cuda_stream), "h2d")
            if fl.size:
                pa.ep_flush = dptr + 4 * o_fl
            pa.n_epochs = len(starts)
            pa.epoch_start, pa.ep_slots, pa.ep_pos = dptr, dptr + 4 * o_es, dptr + 4 * o_pp
            if fabric is not None:
                pa.ep_push, pa.peer_thg = dptr + 4 * o_pm, keep[0].data_ptr()
        _timing.host_stamp("rp:tables")
        tl = None
        if timeline_iters > 0:
            with torch.cuda.stream(self.stream):
                tl = torch.zeros((max(len(slots), 256) + 1, int(timeline_iters), 8), dtype=torch.int64, device=dev)
            pa.timeline, pa.timeline_iters = tl.data_ptr(), int(timeline_iters)
        import time as _time
        if plan is not None:  # temporally blocked kernel: one halo hand-off per k iterations
            ng = int((self.lib.gadmm_chain_blocked_tab_granules_dyn if epochs is not None else
                      self.lib.gadmm_chain_blocked_tab_granules)(self.n_total, self.d, ring))
            if getattr(self, "_blk_tab", None) is None or self._blk_tab.numel() != ng * 4:
                with torch.cuda.stream(self.stream):  # (ordered before the kernel, as _xchk)
                    self._blk_tab = torch.zeros((ng * 4,), dtype=torch.int32, device=dev)
            pa.blk_k, pa.blk_len, pa.blk_pw = plan[0], plan[1], plan[3]
            pa.blk_tab = self._blk_tab.data_ptr()
            if epochs is not None:
                # D-GADMM in the blocked kernel: every inverse as a lane-major image of the kernel's quad
                # register layout (quad_pad_image), reloaded by a re-chain with coalesced unmasked loads
                # (PersistArgs::minv_pad); rebuilt from this solve's inverses on the engine stream, ahead of
                # the launch, only after the inverses changed
                if getattr(self, "_minv_pad", None) is None or self._minv_pad_version != self._minv_version:
                    pf = getattr(self, "_pad_fast", None)
                    if pf is not None and pf[0] is self.Minv and pf[1] is self._minv_pad:
                        native.check(self.lib.gadmm_pad_image_f64(*pf[2]), "pad_image")  # in place, one launch
                    else:
                        with torch.cuda.stream(self.stream):  # in place after the first build (one launch)
                            self._minv_pad = quad_pad_image(self.Minv.reshape(self.n_local * self.nvar, self.d, self.d),
                                                            int(self.lib.gadmm_chain_blocked_pad_dim(self.d)),
                                                            out=getattr(self, "_minv_pad", None))
                        src = _QUAD_SRC.get((self.d, int(self.lib.gadmm_chain_blocked_pad_dim(self.d)), self.device))
                        if src is not None and self.Minv.is_contiguous():
                            # later rebuilds: the same native launch with its arguments bound once
                            self._pad_fast = (self.Minv, self._minv_pad,
                                              (self.Minv.data_ptr(), self.d * self.d, src.data_ptr(), int(src.numel()),
                                               self.n_local * self.nvar, self._minv_pad.data_ptr(),
                                               self.stream.cuda_stream))
                    self._minv_pad_version = self._minv_version
                pa.minv_pad = self._minv_pad.data_ptr()
        self.last_kernel = ("blocked%s(k=%d,L=%d,W=%d,pw=%d)" % ((("-dyn" if epochs is not None else ""),) + tuple(plan))
                            if plan is not None else "per-worker")
        # launches name the engine stream explicitly
        t0 = _time.perf_counter()
        rc = None
        _timing.host_stamp("rp:prelaunch")
        if plan is not None:
            rc = int(self.lib.gadmm_chain_blocked_launch(ctypes.byref(pa), self.stream.cuda_stream))
            _timing.host_stamp("rp:launched")
            if rc == -2 and epochs is None:  # its workgroups cannot all be resident: the per-worker kernel
                plan, rc = None, None
                self.last_kernel = "per-worker"
            else:
                native.check(rc, "chain_blocked_launch")
        if plan is None and self.model == "logistic":
            if epochs is not None:
                raise RuntimeError("persistent logistic kernel: static chains only")
            self._logi = self._logi_args()
            if self.local_solver == "newton":
                self.last_kernel = "per-worker-newton"
                launch = self.lib.gadmm_chain_persistent_newton_launch
            else:
                self.last_kernel = "per-worker-logistic"
                launch = self.lib.gadmm_chain_persistent_logistic_launch
            rc = int(launch(ctypes.byref(pa), ctypes.byref(self._logi), self.stream.cuda_stream))
            if rc == -2:
                raise ResidencyError(self.lib.gadmm_last_error().decode())
            native.check(rc, "chain_persistent_logistic_launch")
        elif plan is None:
            rc = int(self.lib.gadmm_chain_persistent_launch(ctypes.byref(pa), self.stream.cuda_stream))
            if rc == -2:
                raise ResidencyError(self.lib.gadmm_last_error().decode())
            native.check(rc, "chain_persistent_launch")
        # the control block comes back with the same stream sync (pinned buffer, async copy queued
        # behind the kernel): no second blocking round trip per solve
        # the objective trace and the clock come back behind the same sync as the control block, in
        # one copy of the read-back block (short traces: traces() then reads the pinned copy instead of
        # a second blocking device round trip); without them, only the control block's words
        nt = self.trace.numel()
        fetch = fetch_trace and nt <= 16384
        if getattr(self, "_rb_host", None) is None:
            self._rb_host = torch.empty(self._rb.shape, dtype=torch.float64, pin_memory=True)
            self._rb_host_np = self._rb_host.numpy()
            self._ctl_host = self._rb_host[0:4].view(torch.int32)
        # queued on the engine stream (every launch above names that stream explicitly, so no torch stream
        # context is needed around this block) as a small kernel writing the pinned buffer: an SDMA copy
        # started ~10 us after the solve kernel ended (csrc/kernels/readback.hip)
        nb = self._rb.numel() * 8 if fetch else 32  # all of it, or the control block (8 x i32)
        native.check(self.lib.gadmm_readback_d2h(self._rb_host.data_ptr(), self._rb.data_ptr(), nb,
                                                 self.stream.cuda_stream), "readback")
        _timing.host_stamp("rp:copies_queued")
        if on_enqueued is not None:
            on_enqueued()
            _timing.host_stamp("rp:overlapped")
        self.stream.synchronize()
        _timing.host_stamp("rp:synced")
        self._tr_valid = fetch
        t1 = _time.perf_counter()
        self.last_timeline = tl.cpu().numpy() if tl is not None else None
        self.last_timeline_slots = [(s.gid, p) for s, p in zip(slots, pos)] if tl is not None else None
        c = self._ctl_host.tolist()
        done, conv, nxt = c[1], c[2], c[0]
        self.last_placed = c[6]  # ChainCtl::placed: the XCD packing this launch got (0 / 1 / 2)
        if done == 4:
            raise HandoffTimeout("persistent chain kernel timed out (hand-off never completed)")
        # a chunk that ran to its hard stop: count iterations start..hard_stop (only the monitor rank
        # knows the outcome; callers agree on it across ranks)
        last = conv if done in (1, 2, 3) else (int(hard_stop) if hard_stop > 0 else conv)
        p2p = msgs = mon = 0
        if fabric is not None and last >= start_iter:
            # what this rank puts on xGMI for iterations start..conv (the reference's accounting; the
            # lag iterations run past the decision are not counted): theta rows to remote owners of the
            # neighbours, objective granules to the monitor rank, decisions from the monitor rank
            conv_b = last
            ran = conv_b - start_iter + 1
            if epochs is None:
                owner = self._placement_owner
                per_it = sum(len({int(owner[u]) for u in (s.left, s.right) if u >= 0} - {self.rank}) for s in slots)
                msgs = per_it * ran
            else:
                js = np.arange(start_iter, conv_b + 1)
                e_of = np.searchsorted(starts, js, side="right") - 1
                m = mask[e_of]                                                  # (ran, n_local)
                nxt_e = np.minimum(e_of + 1, E - 1)
                starts_next = np.where(e_of + 1 < E, starts[nxt_e], -1)
                m = np.where((js + 1 == starts_next)[:, None], m | mask[nxt_e], m)
                msgs = int(sum(bin(int(v)).count("1") for v in m.reshape(-1)))
            p2p = msgs * self.d * 8
            mon = ran * (len(slots) * 16 if self.rank != 0 else 8 * (self.nranks - 1))
        return EngineRun(conv, done, nxt - start_iter, 1, (t1 - t0) * 1e3, p2p, msgs, mon, 2 * p2p)

    def traces(self, upto: int):
        """(objective trace, measured clock) of iterations 1..upto in ONE device-to-host copy."""
        if upto <= 0:
            return np.zeros((0,), dtype=np.float64), np.zeros((0,), dtype=np.float64)
        if getattr(self, "_tr_valid", False) and upto <= self.trace.numel():  # pinned copy of the last persistent run
            h = self._rb_host_np
            nt = self.trace.numel()
            t = h[8 + nt:8 + nt + upto].view(np.int64)
            tt = (t - int(h[4:5].view(np.int64)[0])) * 1e-8  # (np.where's temporaries: ~2 us per solve)
            tt[t <= 0] = 0.0
            return h[8:8 + upto].copy(), tt
        with torch.cuda.stream(self.stream):
            buf = torch.cat([self.trace[:upto], self.tstamp[:upto].view(torch.float64),
                             self.t0stamp.view(torch.float64)]).cpu().numpy()
        tr = buf[:upto].copy()
        t = buf[upto:2 * upto].view(np.int64)
        t0 = int(buf[2 * upto:].view(np.int64)[0])
        return tr, np.where(t > 0, (t - t0) * 1e-8, 0.0)

    def time_trace(self, upto: int) -> np.ndarray:
        """Measured clock of the last solve: seconds from the solve start (``reset``) to the decision
        of each iteration (s_memrealtime, 100 MHz, stamped by the monitor / the iteration's finish on
        the device). Zero where this rank recorded no decision (non-monitor ranks of the xGMI fabric)."""
        if upto <= 0:
            return np.zeros((0,), dtype=np.float64)
        t = self.tstamp[:upto].cpu().numpy().astype(np.int64)
        t0 = int(self.t0stamp.cpu().item())
        return np.where(t > 0, (t - t0) * 1e-8, 0.0)

    def primal_residual(self, upto: int) -> Optional[np.ndarray]:
        """This rank's part of the K4 primal residual of iterations 1..upto (sum over the chain edges
        whose tail end it owns of ||theta_l - theta||^2 + ||theta - theta_r||^2, summed in worker
        order); None unless the engine was built with ``residual=True``. Ranks' parts add up."""
        if self.rres is None or upto <= 0:
            return None
        return self.rres[: upto * self.n_total].view(upto, self.n_total).cpu().numpy().sum(axis=1)

    def graph_ok(self) -> bool:
        return bool(self.lib.gadmm_chain_engine_graph_ok(self.handle))

    def ctl_state(self) -> dict:
        c = self.ctl.cpu().tolist()
        return {"iter": c[0], "done": c[1], "conv_iter": c[2], "pending": c[3], "ticket": c[4], "monitored": c[5],
                "placed": c[6], "inner_fail": c[7]}

    def objective_trace(self, upto: Optional[int] = None) -> np.ndarray:
        return (self.trace if upto is None else self.trace[:upto]).cpu().numpy()

    def local_theta(self) -> torch.Tensor:
        idx = torch.tensor(self.local_ids, dtype=torch.long, device=self.device)
        return self.theta.index_select(0, idx)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.gadmm_chain_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
