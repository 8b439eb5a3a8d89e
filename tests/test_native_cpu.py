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
           native.PersistArgs.ctl.offset, native.PhaseArgs.lgid.offset, native.EngineDesc.xport.offset,
           native.PersistArgs.xchk.offset, native.PersistArgs.dl_tab.offset, native.PersistArgs.minv_pad.offset,
           native.PersistArgs.ep_flush.offset]
    assert got == exp


def test_fo_abi_layout_matches_ctypes():
    lib = native.require()
    buf = (ctypes.c_longlong * 16)()
    k = lib.gadmm_fo_abi_layout(buf, 16)
    exp = [ctypes.sizeof(native.FoCtl), ctypes.sizeof(native.FoArgs), native.FoArgs.step.offset,
           native.FoArgs.timeout_ticks.offset, native.FoArgs.A.offset, native.FoArgs.ctl.offset,
           native.FoArgs.xchk.offset, native.FoArgs.nranks.offset, native.FoArgs.owner.offset,
           native.FoArgs.pushc.offset]
    assert list(buf[:k]) == exp


def test_code_objects_target_gfx950(tmp_path):
    import shutil
    import subprocess
    # llvm-objdump --offloading extracts every embedded code object NEXT TO its input: run it on a
    # copy in a scratch directory so the in-tree _native/ stays clean
    lib = str(tmp_path / "lib.so")
    shutil.copy(native.library_path(), lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib], capture_output=True,
                         text=True, cwd=str(tmp_path))
    txt = out.stdout + out.stderr
    assert "gfx950" in txt


def test_native_greedy_chains_match_numpy(monkeypatch):
    """csrc/runtime/topology.cpp == PathSchedule's numpy path (findPath / findPath2), bit for bit,
    and == successive step() draws (the reference's one-geometry-per-refresh stream)."""
    import numpy as np
    from gadmm_amd.parallel import topology as T

    native.require()
    for kind in ("findPath2", "findPath"):
        for n in (5, 24, 50):
            s1 = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 10, kind=kind, seed=11)
            P, C = s1.prefetch_arrays(40)
            monkeypatch.setenv("GADMM_NATIVE_TOPOLOGY", "0")
            s2 = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 10, kind=kind, seed=11)
            P2, C2 = s2.prefetch_arrays(40)
            monkeypatch.delenv("GADMM_NATIVE_TOPOLOGY")
            assert np.array_equal(P, P2) and np.array_equal(C, C2)
            s3 = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 10, kind=kind, seed=11)
            for e in range(3):
                s3.step(10 * (e + 1))
                assert s3.path == [int(v) for v in P[e]] and np.array_equal(s3.cost, C[e])
            # skip() == drawing the chains one by one
            s4 = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 10, kind=kind, seed=11)
            s4.skip(s4.save(), P, C, 7)
            s5 = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 10, kind=kind, seed=11)
            s5.prefetch(7)
            assert s4.path == s5.path and np.array_equal(s4.rng.random(4), s5.rng.random(4))
    # a batch large enough for the multi-threaded split (E * n^2 > 400k), with tied distances
    uv = np.random.default_rng(2).random((240, 50, 2))
    uv[:, 7] = uv[:, 3]  # nodes 3 and 7 coincide: the lower index must win every tie
    Pn, Cn = T.native_greedy_chains(uv, 10.0, False)
    xy = uv * 10.0
    dx = xy[:, :, None, 0] - xy[:, None, :, 0]
    dy = xy[:, :, None, 1] - xy[:, None, :, 1]
    d2 = dx * dx + dy * dy
    d2[:, np.arange(50), np.arange(50)] = 0.0
    P = T.greedy_chains(d2)
    assert np.array_equal(Pn, P)
    ar = np.arange(240)[:, None]
    assert np.array_equal(Cn, d2[ar, P[:, :-1], P[:, 1:]])


def test_async_greedy_chains_match_sync():
    """PathSchedule.prefetch_async (geometries from the PCG64 stream and greedy walks on the native host
    worker thread, joined later) == prefetch_arrays: the same chains, costs, current chain and RNG
    position, with the schedule's Generator lazy or materialised; skip() after it; a job never joined is
    drained by the next submit (its buffers stay alive until then)."""
    import numpy as np
    from gadmm_amd.parallel import topology as T

    native.require()
    for kind in ("findPath2", "findPath"):
        s1 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, kind=kind, seed=99)
        P, C = s1.prefetch_arrays(59)
        s2 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, kind=kind, seed=99)
        join = s2.prefetch_async(59)
        assert join is not None
        assert s2.path == list(range(24))  # the current chain moves only at the join
        P2, C2 = join()
        assert np.array_equal(P, P2) and np.array_equal(C, C2)
        assert join()[0] is P2  # idempotent
        assert s1.path == s2.path and np.array_equal(s1.cost, s2.cost)
        assert np.array_equal(s1.rng.random(3), s2.rng.random(3))
    # with the Generator already materialised (and advanced), and after a lazy skip()
    s6 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=7)
    s6.rng.random(5)
    P6, C6 = s6.prefetch_async(11)()
    s7 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=7)
    s7.rng.random(5)
    P7, C7 = s7.prefetch_arrays(11)
    assert np.array_equal(P6, P7) and np.array_equal(C6, C7)
    assert np.array_equal(s6.rng.random(2), s7.rng.random(2))
    s8 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=8)
    sv = s8.save()
    P8, C8 = s8.prefetch_async(9)()
    s8.skip(sv, P8, C8, 4)
    s9 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=8)
    s9.prefetch_arrays(4)
    assert s8.path == s9.path and np.array_equal(s8.rng.random(3), s9.rng.random(3))
    s3 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=5)
    s3.prefetch_async(200)  # dropped without a join
    s4 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=5)
    P4, _ = s4.prefetch_async(3)()
    s5 = T.PathSchedule(24, list(range(24)), np.zeros(23), 10, seed=5)
    assert np.array_equal(P4, s5.prefetch_arrays(3)[0])


def test_native_epoch_tables_match_numpy():
    """csrc/runtime/topology.cpp:gadmm_epoch_tables == the numpy reference (engine/chain_engine.py)."""
    import numpy as np
    from gadmm_amd.ops import native
    from gadmm_amd.engine.chain_engine import epoch_tables_numpy
    lib = native.load(build_if_missing=False)
    rng = np.random.default_rng(3)
    for E, n, loc in ((7, 24, np.arange(24)), (5, 9, np.array([4, 0, 7])), (1, 2, np.array([1]))):
        P = np.ascontiguousarray(np.stack([rng.permutation(n) for _ in range(E)]).astype(np.int64))
        loc = np.ascontiguousarray(loc.astype(np.int64))
        es = np.empty((E * len(loc) * 4,), dtype=np.int32)
        pp = np.empty((E * len(loc),), dtype=np.int32)
        assert lib.gadmm_epoch_tables(P.ctypes.data, E, n, loc.ctypes.data, len(loc), es.ctypes.data,
                                      pp.ctypes.data) == 0
        s_ref, p_ref = epoch_tables_numpy(P, loc)
        assert np.array_equal(es.reshape(E, len(loc), 4), s_ref) and np.array_equal(pp.reshape(E, len(loc)), p_ref)


def test_star_abi_layout_matches_ctypes():
    lib = native.require()
    buf = (ctypes.c_longlong * 8)()
    k = lib.gadmm_star_abi_layout(buf, 8)
    exp = [ctypes.sizeof(native.StarArgs), native.StarArgs.rho.offset, native.StarArgs.gid.offset,
           native.StarArgs.ctl.offset, native.StarArgs.xchk.offset]
    assert list(buf[:k]) == exp


def test_logi_abi_layout_matches_ctypes():
    lib = native.require()
    buf = (ctypes.c_longlong * 8)()
    k = lib.gadmm_logi_abi_layout(buf, 8)
    exp = [ctypes.sizeof(native.LogiArgs), native.LogiArgs.lam.offset, native.LogiArgs.inner_iters.offset]
    assert list(buf[:k]) == exp


def test_blocked_plan_fits_one_xcd():
    """gadmm_chain_blocked_plan: k = 2 and the shortest owned segment whose launch (worker +
    objective + monitor workgroups, one per CU) fits one XCD (32 CUs without a device): N = 24 -> L = 1
    (27 workgroups), N = 50 -> L = 2 (25 + 5 + 1 = 31), N = 100 -> L = 4 (no length fits, the k = 2 maximum)."""
    lib = native.require()
    k, L = ctypes.c_int(0), ctypes.c_int(0)
    for n, want_L in ((24, 1), (50, 2), (8, 1), (100, 4)):
        W = lib.gadmm_chain_blocked_plan(n, 50, 0, ctypes.byref(k), ctypes.byref(L))
        assert (k.value, L.value, W) == (2, want_L, (n + want_L - 1) // want_L), (n, k.value, L.value, W)
    assert lib.gadmm_chain_blocked_plan(24, 100, 0, ctypes.byref(k), ctypes.byref(L)) == 0  # d > 52


def test_epoch_flush_table_matches_the_kernels_old_lookup():
    """PersistArgs::ep_flush (built on the host) == what the blocked D-GADMM kernel used to derive at
    every re-chain from ep_pos / ep_slots: the new worker's old neighbours iff it was an old head."""
    import numpy as np
    from gadmm_amd.engine.chain_engine import epoch_flush_table
    rng = np.random.default_rng(3)
    for E, n in ((1, 5), (6, 9), (11, 24)):
        P = np.stack([rng.permutation(n) for _ in range(E)])
        fl = epoch_flush_table(P)
        pos_of = np.argsort(P, axis=1)
        assert fl.shape == (E, n, 2) and (fl[0] == -1).all()
        for e in range(1, E):
            for p in range(n):
                op = pos_of[e - 1][P[e][p]]
                exp = (P[e - 1][op - 1] if op > 0 else -1, P[e - 1][op + 1] if op < n - 1 else -1) \
                    if op % 2 == 0 else (-1, -1)
                assert tuple(fl[e, p]) == exp


def test_native_blocked_epoch_tables_match_numpy():
    """gadmm_epoch_tables_blocked (C++) == the numpy construction of the blocked D-GADMM tables."""
    import ctypes
    import numpy as np
    from gadmm_amd.engine.chain_engine import epoch_flush_table
    lib = native.require()
    rng = np.random.default_rng(7)
    for E, n in ((1, 4), (9, 24), (40, 7)):
        P = np.ascontiguousarray(np.stack([rng.permutation(n) for _ in range(E)]).astype(np.int64))
        es = np.empty((E * n * 4,), dtype=np.int32)
        pp = np.empty((E * n,), dtype=np.int32)
        fl = np.empty((E * n * 2,), dtype=np.int32)
        assert lib.gadmm_epoch_tables_blocked(P.ctypes.data, E, n, es.ctypes.data, pp.ctypes.data, fl.ctypes.data) == 0
        lft = np.concatenate([np.full((E, 1), -1), P[:, :-1]], axis=1)
        rgt = np.concatenate([P[:, 1:], np.full((E, 1), -1)], axis=1)
        assert np.array_equal(es.reshape(E, n, 4), np.stack([P, P, lft, rgt], axis=-1))
        assert np.array_equal(pp.reshape(E, n), np.argsort(P, axis=1))
        assert np.array_equal(fl.reshape(E, n, 2), epoch_flush_table(P))
    # a row that is not a permutation (duplicate id) is refused by both table builders
    P = np.ascontiguousarray(np.stack([rng.permutation(6), np.array([0, 1, 2, 3, 3, 5])]).astype(np.int64))
    es, pp, fl = (np.empty((2 * 6 * k,), dtype=np.int32) for k in (4, 1, 2))
    assert lib.gadmm_epoch_tables_blocked(P.ctypes.data, 2, 6, es.ctypes.data, pp.ctypes.data, fl.ctypes.data) == -2
    loc = np.arange(6, dtype=np.int64)
    assert lib.gadmm_epoch_tables(P.ctypes.data, 2, 6, loc.ctypes.data, 6, es.ctypes.data, pp.ctypes.data) == -2


def test_quad_pad_image_layout():
    """The lane-major padded inverse image (chain_engine.quad_pad_image) holds, for lane l = i + 16c,
    M[i + 16r, c + 4t] at ((t >> 1) * 4 + r) * 128 + 2 l + (t & 1), and zeros outside d -- the order
    quad_load_image in chain_blocked.hip reads (its per-matrix length is gadmm_chain_blocked_pad_len)."""
    import torch
    from gadmm_amd.engine.chain_engine import quad_pad_image
    from gadmm_amd.ops import native

    for d, db in ((50, 52), (20, 32)):
        M = torch.randn(3, d, d, dtype=torch.float64)
        im = quad_pad_image(M, db)
        assert im.shape == (3, int(native.require().gadmm_chain_blocked_pad_len(d)))
        qt = db // 4
        for b in range(3):
            for t in range(qt):
                for r in range(4):
                    for lane in range(64):
                        row, col = (lane & 15) + 16 * r, (lane >> 4) + 4 * t
                        want = float(M[b, row, col]) if row < d and col < d else 0.0
                        assert float(im[b, ((t >> 1) * 4 + r) * 128 + 2 * lane + (t & 1)]) == want


def test_dl_halo_eligibility_and_heads():
    """The data-local halo mode's plan (engine/blocked_xgmi.py): which boundary heads each rank solves
    and when the mode fits the 12-wave workgroup on every rank (must agree with chain_blocked.hip's
    range hl / hr and the launcher's span check)."""
    from gadmm_amd.engine.blocked_xgmi import dl_halo_eligible, dl_halo_hosted, halo_heads

    def segs(n, world):
        return [(r * n // world, (r + 1) * n // world - 1) for r in range(world)]

    # rank 0: 12 positions + head 12 = 13 waves: the head is hosted by tail 11 (round 4)
    assert dl_halo_eligible(segs(24, 2), 24, 50)
    assert dl_halo_hosted(0, 11, 24) and not dl_halo_hosted(12, 23, 24) and not dl_halo_hosted(6, 11, 24)
    assert not dl_halo_eligible([(0, 12), (13, 23)], 24, 50)  # a 13-position segment never fits
    assert dl_halo_eligible(segs(24, 4), 24, 50)
    assert dl_halo_eligible(segs(24, 8), 24, 50)
    assert not dl_halo_eligible(segs(8, 8), 8, 50)         # one-position segments
    assert not dl_halo_eligible(segs(24, 1), 24, 50)       # one rank: nothing to halo
    assert not dl_halo_eligible(segs(24, 4), 24, 60)       # d > 52
    assert halo_heads(0, 11, 24) == [12] and halo_heads(12, 23, 24) == []  # 2 ranks: 11 is the tail
    assert halo_heads(3, 5, 24) == [2, 6]                  # 8 ranks, rank 1: both edges are tails
    assert halo_heads(0, 2, 24) == [] and halo_heads(6, 8, 24) == []       # heads at the edges
    # every boundary is halo'd by exactly one side
    for world in (4, 8):
        sg = segs(24, world)
        got = sorted(h for lo, hi in sg for h in halo_heads(lo, hi, 24))
        assert len(got) == world - 1 and len(set(got)) == world - 1


def test_star_big_abi_layout_matches_ctypes():
    from gadmm_amd.engine.star_big import StarBigArgs
    lib = native.require()
    buf = (ctypes.c_longlong * 8)()
    k = lib.gadmm_star_big_abi_layout(buf, 8)
    exp = [ctypes.sizeof(StarBigArgs), StarBigArgs.rho.offset, StarBigArgs.Minv.offset, StarBigArgs.ctl.offset,
           StarBigArgs.tstamp.offset, StarBigArgs.gid.offset]
    assert list(buf[:k]) == exp


def test_cg_entry_points_refuse_bad_arguments():
    """The large-d oracle's CG kernels (first_order_big.hip: gadmm_cg_*) validate before launching, so a
    bad call fails loudly on any host (no GPU needed)."""
    lib = native.require()
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.gadmm_cg_begin.restype = ctypes.c_int
    lib.gadmm_cg_begin.argtypes = [P, P, P, P, P, I, P]
    lib.gadmm_cg_resid.restype = ctypes.c_int
    lib.gadmm_cg_resid.argtypes = [P, P, P, I, P]
    assert lib.gadmm_cg_begin(None, None, None, None, None, 10, None) == -1
    assert lib.gadmm_cg_resid(None, None, None, 0, None) == -1
    assert b"cg_" in lib.gadmm_last_error()


def test_epoch_stage_blocked_layout_and_checks():
    """gadmm_epoch_stage_blocked (the D-GADMM launch's fused table staging) writes [starts | slots |
    pos | flush] exactly as gadmm_epoch_tables_blocked builds them and refuses bad starts and
    non-permutations before any copy (here, without a GPU, the final copy itself fails: -3)."""
    import numpy as np

    lib = native.require()
    rng = np.random.default_rng(4)
    E, n = 7, 24
    P = np.ascontiguousarray(np.stack([rng.permutation(n) for _ in range(E)]).astype(np.int64))
    starts = np.arange(1, 1 + 10 * E, 10, dtype=np.int64)
    cap = E + 7 * E * n
    stage = np.zeros(cap, dtype=np.int32)
    rc = lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P.ctypes.data, E, n, 1, 0, stage.ctypes.data, cap,
                                       ctypes.c_void_p(16), None)
    assert rc in (cap, -3)
    es = np.empty(E * n * 4, dtype=np.int32)
    pp = np.empty(E * n, dtype=np.int32)
    fl = np.empty(E * n * 2, dtype=np.int32)
    assert lib.gadmm_epoch_tables_blocked(P.ctypes.data, E, n, es.ctypes.data, pp.ctypes.data, fl.ctypes.data) == 0
    assert np.array_equal(stage, np.concatenate([starts.astype(np.int32), es, pp, fl]))
    bad = starts.copy()
    bad[3] = bad[2]
    assert lib.gadmm_epoch_stage_blocked(bad.ctypes.data, P.ctypes.data, E, n, 1, 0, stage.ctypes.data, cap,
                                         ctypes.c_void_p(16), None) == -1
    assert lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P.ctypes.data, E, n, 2, 0, stage.ctypes.data, cap,
                                         ctypes.c_void_p(16), None) == -1  # first start != start_iter
    assert lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P.ctypes.data, E, n, 2, 1, stage.ctypes.data, cap,
                                         ctypes.c_void_p(16), None) in (cap, -3)  # continuation: at or before
    assert lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P.ctypes.data, E, n, 1, 0, stage.ctypes.data, cap - 1,
                                         ctypes.c_void_p(16), None) == -1  # too small
    P2 = P.copy()
    P2[2, 5] = P2[2, 6]
    assert lib.gadmm_epoch_stage_blocked(starts.ctypes.data, P2.ctypes.data, E, n, 1, 0, stage.ctypes.data, cap,
                                         ctypes.c_void_p(16), None) == -2


def test_fast_getenv_tracks_os_environ(monkeypatch):
    """utils.env.getenv (the hot-path switch reader) == os.environ.get under set / monkeypatch / delete."""
    from gadmm_amd.utils.env import getenv
    monkeypatch.delenv("GADMM_ENV_PROBE", raising=False)
    assert getenv("GADMM_ENV_PROBE") is None and getenv("GADMM_ENV_PROBE", "d") == "d"
    monkeypatch.setenv("GADMM_ENV_PROBE", "7")
    assert getenv("GADMM_ENV_PROBE") == "7"
    os.environ["GADMM_ENV_PROBE"] = "ü"
    assert getenv("GADMM_ENV_PROBE") == os.environ.get("GADMM_ENV_PROBE")
    monkeypatch.delenv("GADMM_ENV_PROBE")
    assert getenv("GADMM_ENV_PROBE", "x") == "x"


def test_xcd_placement_tags_are_fresh_per_launch():
    """PersistArgs::xtag (gadmm_next_xtag): every persistent launch tags its placement-check granules
    with a new value (high bit set: never the memset launchers' XTAG 0x5a5a0001 nor a zeroed granule),
    so granules an earlier launch left in xchk never match and the launcher needs no memset."""
    lib = native.require()
    fn = lib.gadmm_next_xtag
    fn.restype = ctypes.c_uint
    fn.argtypes = []
    tags = [fn() for _ in range(1000)]
    assert len(set(tags)) == len(tags)
    assert all(t & 0x80000000 for t in tags) and 0x5a5a0001 not in tags
    assert all(b == a + 1 for a, b in zip(tags, tags[1:]))
    assert native.PersistArgs.xtag.offset == native.PersistArgs.xcd.offset + 4
