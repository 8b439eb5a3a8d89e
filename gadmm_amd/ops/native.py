"""ctypes binding of ``libgadmm_native.so`` (HIP kernels + C++ runtime for gfx950).

The library has a plain C ABI; tensors are passed as raw device pointers and HIP streams as the
``torch.cuda.Stream.cuda_stream`` handle. ``torch`` is always imported first so the library's
``libamdhip64.so.7`` / ``librccl.so.1`` dependencies bind to the copies torch already loaded (one HIP
runtime per process).

On a machine with a GPU, a missing or stale library is an error (``require()`` raises): GPU code
paths never fall back silently to PyTorch.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (must be loaded before the native library)

_LIB_PATH = os.environ.get("GADMM_NATIVE_LIB") or os.path.join(  # override: A/B runs of two builds
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "libgadmm_native.so")
_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None

c_int, c_long, c_double, c_void_p, c_char_p = ctypes.c_int, ctypes.c_long, ctypes.c_double, ctypes.c_void_p, ctypes.c_char_p
c_longlong = ctypes.c_longlong


class PhaseSlot(ctypes.Structure):
    _fields_ = [("li", c_int), ("gid", c_int), ("left", c_int), ("right", c_int)]


class XchgOp(ctypes.Structure):
    _fields_ = [("peer", c_int), ("row", c_int), ("is_send", c_int), ("count", c_int)]


class ChainCtl(ctypes.Structure):
    _fields_ = [("iter", c_int), ("done", c_int), ("conv_iter", c_int), ("pending", c_int),
                ("ticket", ctypes.c_uint), ("monitored", c_int), ("pad", c_int * 2)]


class PhaseArgs(ctypes.Structure):
    _fields_ = [
        ("d", c_int), ("n_slots", c_int), ("n_local", c_int), ("nvar", c_int),
        ("deg_to_var", c_int * 3),
        ("flags", c_int), ("model", c_int),
        ("slots", c_void_p), ("Minv", c_void_p), ("A", c_void_p), ("b", c_void_p), ("yy", c_void_p),
        ("mu", c_void_p), ("theta", c_void_p),
        ("rho", c_double),
        ("objw", c_void_p), ("ctl", c_void_p), ("trace", c_void_p), ("part", c_void_p),
        ("ring", c_int), ("max_iter", c_int),
        ("obj0", c_double), ("tol", c_double),
        ("X", c_void_p), ("Y", c_void_p),
        ("m", c_int), ("max_inner", c_int),
        ("lam", c_double), ("step", c_double), ("inner_tol", c_double),
        ("inner_iters", c_void_p),
        ("rbuf", c_void_p), ("obj_mode", c_int), ("solver", c_int),
        ("n_total", c_int), ("pad_nt", c_int), ("lgid", c_void_p), ("tstamp", c_void_p),
        ("rres", c_void_p),
    ]


class EngineDesc(ctypes.Structure):
    _fields_ = [("base", PhaseArgs), ("d_slots", c_void_p), ("reduced", c_void_p), ("comm", c_void_p),
                ("stream", c_void_p), ("nranks", c_int), ("xport", c_void_p)]


class FoCtl(ctypes.Structure):
    _fields_ = [("monitored", c_int), ("stop_iter", c_int), ("status", c_int), ("iters", c_int),
                ("uploads", c_double), ("pad_", c_double)]


class FoArgs(ctypes.Structure):
    """Mirror of csrc/include/gadmm_fo.h (persistent first-order baseline engine)."""
    _fields_ = [
        ("alg", c_int), ("model", c_int), ("n", c_int), ("d", c_int), ("m", c_int), ("max_iter", c_int),
        ("faithful", c_int), ("jacobi", c_int), ("has_tol", c_int), ("ring", c_int),
        ("epoch", ctypes.c_uint), ("slots", c_int),
        ("step", c_double), ("lam", c_double), ("obj0", c_double), ("tol", c_double), ("thrd", c_double),
        ("timeout_ticks", c_longlong),
        ("A", c_void_p), ("b", c_void_p), ("yy", c_void_p), ("X", c_void_p), ("Y", c_void_p),
        ("hsq", c_void_p), ("sched", c_void_p), ("tab", c_void_p), ("part", c_void_p),
        ("obj_trace", c_void_p), ("cnt_trace", c_void_p), ("time_trace", c_void_p), ("theta_out", c_void_p),
        ("ctl", c_void_p), ("xchk", c_void_p), ("xcd", c_int), ("pad_x", c_int),
        ("nranks", c_int), ("my_rank", c_int), ("w_lo", c_int), ("n_local", c_int),
        ("has_monitor", c_int), ("pad_m", c_int),
        ("owner", c_void_p), ("tab_push", c_void_p), ("wmon", c_void_p), ("wstop", c_void_p),
        ("wpush", c_void_p), ("pushc", c_void_p),
    ]


class RunStats(ctypes.Structure):
    _fields_ = [("iters", c_int), ("done", c_int), ("iterations_launched", c_int), ("replays", c_int),
                ("wall_ms", c_double), ("p2p_bytes", c_longlong), ("p2p_msgs", c_longlong),
                ("monitor_bytes", c_longlong), ("wire_bytes", c_longlong)]


class PersistArgs(ctypes.Structure):
    _fields_ = [
        ("d", c_int), ("n", c_int), ("n_local", c_int), ("start_iter", c_int), ("max_iter", c_int),
        ("lag", c_int), ("ring", c_int), ("nvar", c_int), ("obj_mode", c_int), ("deg_to_var", c_int * 3),
        ("pending_in", c_int), ("has_monitor", c_int), ("nranks", c_int), ("sys_scope", c_int),
        ("epoch", ctypes.c_uint), ("blk_pw", c_int),
        ("rho", c_double), ("obj0", c_double), ("tol", c_double), ("timeout_ticks", c_longlong),
        ("slots", c_void_p), ("pos", c_void_p), ("Minv", c_void_p), ("A", c_void_p), ("b", c_void_p),
        ("yy", c_void_p), ("theta", c_void_p), ("mu", c_void_p), ("thg", c_void_p), ("push", c_void_p),
        ("objg", c_void_p), ("decg", c_void_p), ("dec_push", c_void_p), ("trace", c_void_p), ("ctl", c_void_p),
        ("timeline", c_void_p), ("timeline_iters", c_int), ("blk_k", c_int), ("blk_len", c_int), ("n_epochs", c_int),
        ("blk_tab", c_void_p), ("epoch_start", c_void_p), ("ep_slots", c_void_p), ("ep_pos", c_void_p),
        ("seg_lo", c_int), ("seg_hi", c_int), ("blk_npeer", c_int), ("dbg", c_int),
        ("blk_peer_lo", c_int * 8), ("blk_peer_hi", c_int * 8), ("blk_peer_tab", c_void_p),
        ("tstamp", c_void_p), ("ep_push", c_void_p), ("peer_thg", c_void_p), ("rres", c_void_p),
        ("hard_stop", c_int), ("cont", c_int),
        ("xchk", c_void_p), ("xcd", c_int), ("xtag", c_int),
        ("blk_dl", c_int), ("dl_halo", c_int), ("dl_tab", c_void_p * 2), ("minv_pad", c_void_p),
        ("ep_flush", c_void_p),
    ]


class LogiArgs(ctypes.Structure):
    """Mirror of LogiArgs in csrc/kernels/chain_persistent_logistic.hip (persistent logistic GADMM)."""
    _fields_ = [("X", c_void_p), ("Y", c_void_p), ("m", c_int), ("max_inner", c_int),
                ("lam", c_double), ("step", c_double), ("inner_tol", c_double), ("inner_iters", c_void_p),
                ("scratch", c_void_p)]


class StarArgs(ctypes.Structure):
    """Mirror of csrc/include/gadmm_star.h (persistent star ADMM)."""
    _fields_ = [
        ("d", c_int), ("n", c_int), ("n_local", c_int), ("max_iter", c_int),
        ("lag", c_int), ("ring", c_int), ("has_monitor", c_int), ("nranks", c_int),
        ("sys_scope", c_int), ("hub_rank", c_int), ("my_rank", c_int), ("timeline_iters", c_int),
        ("epoch", ctypes.c_uint), ("pad1", c_int),
        ("rho", c_double), ("obj0", c_double), ("tol", c_double), ("timeout_ticks", c_longlong),
        ("gid", c_void_p), ("Minv", c_void_p), ("A", c_void_p), ("b", c_void_p), ("yy", c_void_p),
        ("theta", c_void_p), ("lam", c_void_p), ("lam_hub", c_void_p), ("thg", c_void_p), ("peer_thg", c_void_p),
        ("objg", c_void_p), ("decg", c_void_p), ("dec_push", c_void_p), ("trace", c_void_p), ("tstamp", c_void_p),
        ("ctl", c_void_p), ("timeline", c_void_p), ("xchk", c_void_p), ("xcd", c_int), ("pad2", c_int),
    ]


MODEL_LINEAR, MODEL_LOGISTIC = 0, 1


def _declare(lib: ctypes.CDLL) -> None:
    sig = {
        "gadmm_last_error": (c_char_p, []),
        "gadmm_native_version": (c_int, []),
        "gadmm_device_info": (c_int, [c_int, c_char_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_longlong),
                                      ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
        "gadmm_gram_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
        "gadmm_gram_workspace": (c_long, [c_int, c_int, c_int, c_int]),
        "gadmm_gram_pick_ksplit": (c_int, [c_int, c_int, c_int]),
        "gadmm_spd_inverse_small_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                                c_void_p]),
        "gadmm_spd_inverse_blocked_workspace": (c_long, [c_int, c_int]),
        "gadmm_spd_inverse_blocked_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                                  c_void_p, c_int, c_void_p]),
        "gadmm_gemm_f64_test": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
        "gadmm_chain_phase": (c_int, [ctypes.POINTER(PhaseArgs), c_void_p]),
        "gadmm_chain_reset": (c_int, [c_void_p, c_int, c_int, c_void_p]),
        "gadmm_chain_reset_state": (c_int, [c_void_p, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p,
                                            c_long, c_void_p, c_long, c_void_p]),
        "gadmm_chain_reset_state_stamp": (c_int, [c_void_p, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p,
                                            c_long, c_void_p, c_long, c_void_p, c_void_p]),
        "gadmm_chain_engine_create": (c_void_p, [ctypes.POINTER(EngineDesc)]),
        "gadmm_chain_engine_destroy": (None, [c_void_p]),
        "gadmm_chain_engine_set_plan": (c_int, [c_void_p, c_int, ctypes.POINTER(PhaseSlot), c_int,
                                                ctypes.POINTER(PhaseSlot), c_int, ctypes.POINTER(XchgOp), c_int,
                                                ctypes.POINTER(XchgOp)]),
        "gadmm_chain_engine_set_scalars": (c_int, [c_void_p, c_double, c_double, c_double, c_int]),
        "gadmm_chain_engine_reset": (c_int, [c_void_p, c_int, c_int]),
        "gadmm_chain_engine_flush": (c_int, [c_void_p]),
        "gadmm_chain_engine_run": (c_int, [c_void_p, c_int, c_int, c_int, ctypes.POINTER(RunStats)]),
        "gadmm_chain_engine_graph_ok": (c_int, [c_void_p]),
        "gadmm_chain_engine_exchange": (c_int, [c_void_p, c_int]),
        "gadmm_abi_layout": (c_int, [ctypes.POINTER(c_longlong), c_int]),
        "gadmm_chain_persistent_lds": (c_long, [c_int, c_int]),
        "gadmm_chain_persistent_lds_dyn": (c_long, [c_int, c_int, c_int]),
        "gadmm_chain_big_rbuf_stride": (c_long, [c_int]),
        "gadmm_xgmi_alloc": (c_int, [ctypes.c_size_t, ctypes.POINTER(c_void_p), ctypes.c_char_p]),
        "gadmm_xgmi_open": (c_int, [ctypes.c_char_p, ctypes.POINTER(c_void_p)]),
        "gadmm_xgmi_close": (c_int, [c_void_p]),
        "gadmm_xgmi_free": (c_int, [c_void_p]),
        "gadmm_device_can_access_peer": (c_int, [c_int, c_int]),
        "gadmm_chain_persistent_launch": (c_int, [ctypes.POINTER(PersistArgs), c_void_p]),
        "gadmm_chain_persistent_capacity": (c_long, [ctypes.POINTER(PersistArgs)]),
        "gadmm_chain_persistent_logistic_capacity": (c_long, [ctypes.POINTER(PersistArgs), ctypes.POINTER(LogiArgs)]),
        "gadmm_chain_persistent_logistic_launch": (c_int, [ctypes.POINTER(PersistArgs), ctypes.POINTER(LogiArgs),
                                                           c_void_p]),
        "gadmm_logi_abi_layout": (c_int, [ctypes.POINTER(c_longlong), c_int]),
        "gadmm_chain_persistent_newton_capacity": (c_long, [ctypes.POINTER(PersistArgs), ctypes.POINTER(LogiArgs)]),
        "gadmm_newton_rec_scratch_doubles": (c_long, []),
        "gadmm_chain_persistent_newton_launch": (c_int, [ctypes.POINTER(PersistArgs), ctypes.POINTER(LogiArgs),
                                                         c_void_p]),
        "gadmm_write_stamp": (c_int, [c_void_p, c_void_p]),
        "gadmm_star_capacity": (c_long, [ctypes.POINTER(StarArgs)]),
        "gadmm_star_launch": (c_int, [ctypes.POINTER(StarArgs), c_void_p]),
        "gadmm_star_abi_layout": (c_int, [ctypes.POINTER(c_longlong), c_int]),
        "gadmm_star_big_abi_layout": (c_int, [ctypes.POINTER(c_longlong), c_int]),
        "gadmm_sym_pack_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
        "gadmm_sym_packed_doubles": (c_long, [c_int]),
        "gadmm_ipc_box_bytes": (c_long, [c_int, c_int, c_int, c_int]),
        "gadmm_ipc_collective": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, ctypes.c_uint, c_void_p,
                                         c_void_p]),
        "gadmm_ipc_coll_counters": (c_int, [c_void_p, ctypes.POINTER(c_longlong)]),
        "gadmm_ipc_hop_probe": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_uint, c_double,
                                        ctypes.POINTER(ctypes.c_ulonglong)]),
        "gadmm_ipc_xport_create": (c_void_p, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_double]),
        "gadmm_ipc_xport_destroy": (c_int, [c_void_p]),
        "gadmm_ipc_new_epoch": (c_int, [c_void_p, c_void_p]),
        "gadmm_ipc_counters": (c_int, [c_void_p, ctypes.POINTER(c_longlong)]),
        "gadmm_chain_blocked_plan": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
        "gadmm_chain_blocked_plan2": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                              ctypes.POINTER(c_int)]),
        "gadmm_chain_blocked_lds": (c_long, [c_int, c_int]),
        "gadmm_chain_blocked_plan_dl": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
        "gadmm_chain_blocked_pad_dim": (c_int, [c_int]),
        "gadmm_chain_blocked_pad_len": (c_long, [c_int]),
        "gadmm_chain_blocked_max_epochs": (c_int, []),
        "gadmm_memcpy_h2d_async": (c_int, [c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
        "gadmm_memcpy_d2h_async": (c_int, [c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
        "gadmm_readback_d2h": (c_int, [c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
        "gadmm_chain_blocked_tab_granules": (c_long, [c_int, c_int, c_int]),
        "gadmm_chain_blocked_tab_granules_dyn": (c_long, [c_int, c_int, c_int]),
        "gadmm_epoch_tables": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p]),
        "gadmm_epoch_tables_blocked": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
        "gadmm_epoch_stage_blocked": (c_long, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_long,
                                               c_void_p, c_void_p]),
        "gadmm_chain_blocked_launch": (c_int, [ctypes.POINTER(PersistArgs), c_void_p]),
        "gadmm_fo_lds": (c_long, [c_int, c_int, c_int, c_int, c_int]),
        "gadmm_fo_tab_granules": (c_long, [c_int, c_int, c_int]),
        "gadmm_fo_abi_layout": (c_int, [ctypes.POINTER(c_longlong), c_int]),
        "gadmm_fo_launch": (c_int, [ctypes.POINTER(FoArgs), c_void_p]),
        "gadmm_quad_gemv_test": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
        "gadmm_greedy_chains": (c_int, [c_void_p, c_int, c_int, c_double, c_int, c_double, c_double, c_double,
                                        c_void_p, c_void_p]),
        "gadmm_greedy_chains_async": (c_int, [c_void_p, c_int, c_int, c_double, c_int, c_double, c_double,
                                              c_double, c_void_p, c_void_p]),
        "gadmm_greedy_chains_wait": (c_int, []),
        "gadmm_pcg64_uniform": (c_int, [ctypes.c_ulonglong] * 5 + [c_long, c_void_p]),
        "gadmm_draw_chains_async": (c_int, [ctypes.c_ulonglong] * 5 + [c_void_p, c_int, c_int, c_double, c_int, c_double,
                                                                        c_double, c_double, c_void_p, c_void_p]),
        "gadmm_rccl_unique_id": (c_int, [ctypes.c_char_p]),
        "gadmm_rccl_version": (c_int, []),
        "gadmm_rccl_init": (c_void_p, [ctypes.c_char_p, c_int, c_int, c_int]),
        "gadmm_rccl_init_timeout": (c_void_p, [ctypes.c_char_p, c_int, c_int, c_int, ctypes.c_double]),
        "gadmm_rccl_set_timeout": (c_int, [c_void_p, ctypes.c_double]),
        "gadmm_rccl_alive": (c_int, [c_void_p]),
        "gadmm_rccl_abort": (c_int, [c_void_p]),
        "gadmm_rccl_wait": (c_int, [c_void_p, c_void_p, ctypes.c_double]),
        "gadmm_debug_busy_wait": (c_int, [ctypes.c_double, c_void_p]),
        "gadmm_gram_ozaki_workspace": (c_long, [c_long, c_int]),
        "gadmm_gram_crt_workspace": (c_long, [c_long, c_int]),
        "gadmm_gram_crt_max_rows": (c_long, []),
        "gadmm_gram_crt_f64": (c_int, [c_void_p, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_long, c_void_p, c_void_p]),
        "gadmm_gram_ozaki_f64": (c_int, [c_void_p, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_long, c_void_p, c_void_p]),
        "gadmm_chain_engine_set_timeout": (c_int, [c_void_p, ctypes.c_double]),
        "gadmm_rccl_destroy": (c_int, [c_void_p]),
        "gadmm_rccl_exchange_rows": (c_int, [c_void_p, ctypes.POINTER(XchgOp), c_int, c_void_p, c_int, c_void_p]),
        "gadmm_rccl_allreduce_sum_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_void_p]),
        "gadmm_rccl_reduce_sum_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
        "gadmm_rccl_bcast_f64": (c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p]),
        "gadmm_rccl_counters": (c_int, [c_void_p, ctypes.POINTER(c_longlong)]),
        "gadmm_rccl_reset_counters": (c_int, [c_void_p]),
        "gadmm_poison_lds": (c_int, [c_long, c_int, c_void_p]),
        "gadmm_poison_buffer": (c_int, [c_void_p, c_long, c_void_p]),
        "gadmm_lds_probe": (c_int, [c_void_p, c_int, c_int, c_void_p]),
        "gadmm_memset_async": (c_int, [c_void_p, c_int, c_long, c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def library_path() -> str:
    return _LIB_PATH


def load(build_if_missing: bool = True) -> Optional[ctypes.CDLL]:
    """Load (building first when missing/stale and a toolchain is available)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    try:
        if build_if_missing:
            from .. import _build
            try:
                _build.build(verbose=False)
            except Exception as e:  # toolchain missing: fine if a built library exists
                if not os.path.exists(_LIB_PATH):
                    raise RuntimeError("native build failed: %s" % e)
        lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(lib)
        _lib = lib
    except Exception as e:  # pragma: no cover - depends on the box
        _load_error = str(e)
        _lib = None
    return _lib


def available() -> bool:
    return load() is not None


def require() -> ctypes.CDLL:
    lib = load()
    if lib is None:
        raise RuntimeError("gadmm_amd native library unavailable (%s): build it with "
                           "`python -m gadmm_amd._build`" % _load_error)
    return lib


RCCL_DEAD = -77  # csrc/include/gadmm_common.h: GADMM_RCCL_DEAD


class RcclDead(RuntimeError):
    """An RCCL communicator's watchdog deadline passed (or RCCL reported an asynchronous error): the
    communicator was aborted and refuses further calls; the caller falls back to another data plane."""


class NativeTimeout(RuntimeError):
    """A bounded host wait of the native engine passed its deadline (a stalled peer or collective)."""


ENGINE_TIMEOUT = -78  # csrc/runtime/chain_engine.cpp: a bounded wait passed its deadline
RCCL_WEDGED = -79     # a watchdog abort after which the stream did not drain


class DeviceWedged(SystemExit):
    """The device stream did not drain after a watchdog abort: no fallback may run on this device.
    A SystemExit (not caught by the ``except RuntimeError`` fallbacks): the process exits non-zero."""


def check(rc: int, what: str = "native call") -> None:
    if rc != 0:
        msg = require().gadmm_last_error()
        text = "%s failed (rc=%d): %s" % (what, rc, msg.decode() if msg else "?")
        if rc == RCCL_DEAD:
            raise RcclDead(text)
        if rc == ENGINE_TIMEOUT:
            raise NativeTimeout(text)
        if rc == RCCL_WEDGED:
            import sys
            print("gadmm_amd: " + text, file=sys.stderr, flush=True)
            raise DeviceWedged(5)
        raise RuntimeError(text)


def poison_lds(per_cu: int = 4, sync: bool = True) -> None:
    """Fill every CU's LDS with NaN patterns (csrc/kernels/debug_poison.hip). A kernel that reads
    LDS it did not write then produces NaN deterministically instead of depending on what the
    previous kernel left behind (the GPU test tier poisons before every test)."""
    check(require().gadmm_poison_lds(0, per_cu, stream_handle()), "poison_lds")
    if sync:
        torch.cuda.synchronize()


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
