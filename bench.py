"""Headline benchmark: wall-clock and communication bytes to a 1e-8 objective gap (BASELINE.json).

Config (BASELINE.json configs[1], BASELINE.md "GADMM lin-syn iterations to 1e-8"): the
LinearRegression_Synthetic problem of the reference -- N = 24 logical workers (``--workers``), d = 50
features, m = 50 samples per worker, X_n = 1.3^(n-1) q_n q_n^T + I (rebuilt from the reference's
shipped inputData.mat), closed-form local solves, GADMM with rho = 3, stop at |obj - obj0| < 1e-8.
``--workers 8`` is configs[1] literally: 8 workers, so on 8 GPUs each MI355X is one worker.

The workers form one chain laid over the GPUs in contiguous segments. **Data-local by default**: a
rank builds and holds only its own workers' shards (``benchmarks.headline_rank_problem``) and ships
only theta, to the two chain neighbours (group_ADMM_closedForm.m:18-27, 62-70):
* 1 GPU: the temporally blocked persistent kernel (one launch per solve);
* N GPUs (``--fabric auto``/``xgmi``): the temporally blocked kernel run inside every rank's segment
  (data-local mode: only the segment-edge workers' theta crosses, every phase, pushed into the
  neighbour GPU's ring over xGMI -- device-initiated, IPC-mapped fine-grained memory). When every
  segment has >= 2 workers (N <= 12 GPUs at 24 workers) it runs in the one-position halo mode: at each
  rank boundary the rank holding the tail also solves the other rank's boundary head (its 20 KB shard
  is fetched once and reported as replicated_shard_bytes, data_local then reads false), so each
  iteration carries one cross-GPU hop on the critical cycle instead of two (GADMM_DL_HALO=0: off);
  if the blocked kernel is unavailable, the per-worker persistent kernel over the same fabric;
* fallbacks, taken by every rank together: the graph-replayed phase kernels with RCCL send/recv
  (``--fabric rccl``), or with the device-copy transport (``--fabric ipc``; also the fallback when
  ranks share one GPU, where RCCL cannot run).
``--engine replicated-halo`` is the opt-in temporally blocked kernel across GPUs: each rank ALSO holds
the shards of a 4-position halo of other ranks' workers and exchanges (theta, mu) once per 2
iterations; its replicated shard bytes are reported.

One *step* = one complete solve from the raw shards already resident on the GPU: Gram + b + y^T y
(f64 MFMA), cached inverses, then GADMM iterations from theta = mu = 0 until the device-side stop
rule fires. Every timed step must converge in the reference's iteration count (1373 at rho = 3,
N = 24). Bytes per solve are reported three ways, summed over ranks: theta payload (8 B per double),
wire (the xGMI / IPC granules carry 16 B per double) and stop-rule monitor traffic.
``value`` is seconds per solve (lower is better); ``vs_baseline`` = value / 1.13 s, the CPU wall time
of the same loop ([measured-here] row).

    python bench.py                      # 1 GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

The other BASELINE.json configs (same JSON contract, own metric): ``--config cpu_gloo`` (configs[0]: the
same GADMM over gloo CPU ranks, no GPU), ``--config logistic`` (configs[2]), ``--config dgadmm``
(configs[3]), ``--config real10m`` (configs[4]: 1.25M x 10k f64 per GPU), ``--config star`` (the
star-ADMM comparator of E7); see gadmm_amd/benchmarks.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_S = 1.13  # CPU wall time of the GADMM loop to 1e-8, rho = 3


class BenchFailure(RuntimeError):
    pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rho", type=float, default=3.0)
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--workers", type=int, default=24)
    ap.add_argument("--block", type=int, default=0, help="iterations per graph replay (0: auto)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--engine", choices=["auto", "persistent", "blocked-dl", "per-worker", "graph", "replicated-halo"],
                    default="auto",
                    help="auto: one GPU = the persistent single-launch kernel; N GPUs = an engine tournament in "
                         "the untimed warm-up (data-local blocked with / without its halo mode, per-worker, "
                         "replicated-halo: each timed, the fastest agreed by all ranks), the graph engine if "
                         "none runs; blocked-dl / per-worker: only that persistent kernel; replicated-halo: "
                         "opt-in blocked kernel across GPUs (ranks hold halo shards)")
    ap.add_argument("--fabric", choices=["auto", "xgmi", "rccl", "ipc"], default="auto",
                    help="multi-GPU transport: xgmi = device-initiated theta pushes between persistent kernels, "
                         "rccl = RCCL send/recv between graph-replayed phases, ipc = the device-copy transport "
                         "between graph-replayed phases")
    ap.add_argument("--config", choices=["e1", "logistic", "logistic_exact", "dgadmm", "real10m", "star", "cpu_gloo"],
                    default="e1", help="e1 = the headline (default); the others are BASELINE.json configs[2..4]; "
                                       "cpu_gloo = configs[0]: the same GADMM over gloo ranks on the CPU (plumbing, "
                                       "no GPU; launch with torchrun --nproc-per-node 2)")
    ap.add_argument("--coherence", type=int, default=10,
                    help="dgadmm: iterations between re-chains (1 = BASELINE configs[3]'s 're-chaining each round')")
    ap.add_argument("--rows", type=int, default=1_250_000, help="real10m: rows per GPU")
    ap.add_argument("--dim", type=int, default=10_000, help="real10m: features")
    ap.add_argument("--timeout", type=float, default=20.0,
                    help="multi-GPU hand-off deadline in seconds (a stalled peer ends a solve with done=4)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == "cpu_gloo":  # BASELINE configs[0]: no device is touched
        run_cpu_gloo(args, rank, world)
        return
    if world != args.gpus and world == 1 and args.gpus > 1:
        print("bench.py: --gpus %d needs a torchrun launch with %d processes" % (args.gpus, args.gpus),
              file=sys.stderr)
        sys.exit(2)
    # GADMM_BENCH_SHARE_GPU=1: rehearsal of the multi-rank path with every rank on cuda:0 (one-GPU
    # development box). RCCL refuses two ranks on one device, so there the fallback is the IPC transport.
    from gadmm_amd.parallel.node import select_device_index, share_requested
    share = share_requested()
    # local_rank % visible devices: every GPU visible -> rank r on device r; a per-process
    # HIP_VISIBLE_DEVICES (one visible device) -> device 0 (counting devices does not initialise HIP)
    dev_index = select_device_index(local_rank, share, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if args.config != "e1":
            run_other(args, rank, world, device, share)
        else:
            run_headline(args, rank, world, device, share)
    except BenchFailure as e:
        print("bench.py[rank %d]: FAILED: %s" % (rank, e), file=sys.stderr, flush=True)
        sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


# Per-iteration cost of each engine family's kernel on ONE MI355X with no cross-GPU hop (measured:
# profiles/r04_final e1 1.755 ms / 1373 for the blocked layout, README per-worker 3.07 ms / 1373, the
# paired layout 2.80 ms / 1373 in profiles/r01c_pair_layout): the compute term of the tournament's model
# predicted_ms = iters x (one_gpu_us + hops_per_iter x xgmi_hop_us) / 1e3.
ONE_GPU_US = {"blocked": 1.28, "per-worker": 2.24, "paired": 2.04}


def _one_gpu_calibration(args, rank, world, device, obj0):
    """The compute term of the tournament's model measured on THIS box (the
    ONE_GPU_US constants come from other boxes' profiles): rank 0 times the whole chain on its own GPU
    on the one-GPU temporally blocked kernel (3 solves after 2 warm ones; the other ranks wait at the
    broadcast, so a shared GPU is not time-shared meanwhile) and every rank gets the microseconds per
    iteration. 0 / None when it fails (the constants are used then)."""
    us = 0.0
    if rank == 0:
        try:
            from gadmm_amd.data import linear_synthetic
            from gadmm_amd.models import LinearRegression
            from gadmm_amd.algorithms import chain_admm
            ds = linear_synthetic(args.workers)
            mdl = LinearRegression(ds.X.to(device).contiguous(), ds.y.to(device).contiguous())
            ids = list(range(args.workers))

            def solve():
                return chain_admm(mdl, ids, args.workers, args.rho, obj0, args.tol, 3000,
                                  engine_opts={"state": False, "residual": False})
            for _ in range(2):
                solve()
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            for _ in range(3):
                r = solve()
            torch.cuda.synchronize(device)
            if r.extra.get("engine") == "persistent" and r.iters > 0:
                us = (time.perf_counter() - t0) / 3 * 1e6 / r.iters
            del mdl
        except Exception as e:  # the model falls back to the constants
            print("bench.py: one-GPU calibration failed: %s" % e, file=sys.stderr, flush=True)
            us = 0.0
    t = torch.tensor([us], dtype=torch.float64)
    dist.broadcast(t, src=0)
    return float(t.item()) or None


def _headline_candidates(args, X_cpu, y_cpu, local, placement, rank, world, device, share, obj0):
    """Every multi-GPU engine the tournament times, in preference order: dicts with ``name``, ``build``
    (timeout_s -> solver; collective), ``hops`` (cross-GPU hand-offs on the critical cycle per iteration,
    group_ADMM_closedForm.m:18-27, 62-70: the data-local kernel pays head -> tail -> head = 2, its halo
    mode 1, the replicated-halo kernel 1 per k iterations) and ``base`` (its ONE_GPU_US family)."""
    from gadmm_amd.engine.multigpu import DistributedChainSolver

    def make(engine, fabric=None, **kw):
        def build(timeout_s):
            sol = DistributedChainSolver(X_cpu.to(device).contiguous(), y_cpu.to(device).contiguous(), local,
                                         args.workers, placement, rank, world, device, args.rho, obj0, args.tol,
                                         engine=engine, fabric=fabric or args.fabric, share=share,
                                         block=args.block, use_graph=not args.no_graph, timeout_s=timeout_s,
                                         strict=True, **kw)
            if fabric is not None and engine == "graph" and sol.kind != fabric:  # e.g. RCCL fell back to IPC
                got = sol.kind
                sol.close()
                raise RuntimeError("graph engine over %s unavailable (got %s)" % (fabric, got))
            return sol
        return build

    def replicated(k, pw):
        def build(timeout_s):
            from gadmm_amd.data import linear_synthetic
            ds_all = linear_synthetic(args.workers)  # the halo engine holds other ranks' shards (reported)
            return make("replicated-halo", halo_data=(ds_all.X, ds_all.y), halo_k=k, halo_pw=pw)(timeout_s)
        return build

    cands = []
    if args.fabric in ("auto", "xgmi"):
        cands += [dict(name="blocked-dl-halo", build=make("blocked-dl", dl_halo=True), hops=1.0, base="blocked"),
                  dict(name="blocked-dl", build=make("blocked-dl", dl_halo=False), hops=2.0, base="blocked"),
                  dict(name="per-worker", build=make("per-worker"), hops=2.0, base="per-worker")]
        from gadmm_amd.engine.blocked_xgmi import replicated_plans
        for k, pw in replicated_plans(args.workers, placement, int(X_cpu.shape[2])):
            cands.append(dict(name="replicated-halo-k%d%s" % (k, "-pw2" if pw == 2 else ""), build=replicated(k, pw),
                              hops=1.0 / k, base="paired" if pw == 2 else "blocked"))
    if os.environ.get("GADMM_TOURNAMENT_GRAPH", "1") != "0":
        # the graph-replayed phase kernels over the node's default data plane, the IPC transport
        # (measured, never expected to win). RCCL (graph-rccl) only on request -- GADMM_TOURNAMENT_RCCL=1
        # or --fabric rccl, on distinct GPUs: the default run builds no RCCL communicator at all
        cands.append(dict(name="graph-ipc", build=make("graph", fabric="ipc"), hops=2.0, base=None))
        if not share and (args.fabric == "rccl" or os.environ.get("GADMM_TOURNAMENT_RCCL") == "1"):
            cands.append(dict(name="graph-rccl", build=make("graph", fabric="rccl"), hops=2.0, base=None))
    return cands


def run_headline(args, rank, world, device, share):
    from gadmm_amd.benchmarks import headline_rank_problem, EXPECTED_ITERS_1E8
    from gadmm_amd.engine.multigpu import DistributedChainSolver, all_ok
    from gadmm_amd.parallel.topology import chain_message_count

    X_cpu, y_cpu, local, placement, obj0 = headline_rank_problem(args.workers, rank, world)
    d, m = int(X_cpu.shape[2]), int(X_cpu.shape[1])
    expect = EXPECTED_ITERS_1E8.get((args.workers, float(args.rho))) if args.tol == 1e-8 else None
    timeout_s = float(args.timeout)
    tour_timeout_s = min(timeout_s, 5.0)
    hop = None
    if world > 1:
        # one-way hop latency of every chain boundary (the quantity that decides the engine ranking)
        from gadmm_amd.parallel.hop_probe import hop_probe
        hop = hop_probe(rank, world, device)
    sol, tournament, winner, tour_wall_s, calib_us = None, None, None, None, None
    if world > 1 and args.engine == "auto":
        # untimed: build and time every eligible multi-GPU engine, agree on the fastest (max over ranks).
        # A candidate that stalls (e.g. a persistent kernel whose peers cannot be co-resident with ranks
        # time-sharing one GPU) fails within the tournament's 5 s deadline instead of the full one; the
        # winner is then REBUILT with the requested --timeout for the warm-up and the timed solves.
        from gadmm_amd.engine.tournament import engine_tournament
        t_tour = time.perf_counter()
        cands = _headline_candidates(args, X_cpu, y_cpu, local, placement, rank, world, device, share, obj0)
        log = (lambda msg: print("bench.py: " + msg, file=sys.stderr, flush=True)) if rank == 0 else None
        winner, sol, tournament = engine_tournament([(c["name"], (lambda b=c["build"]: b(tour_timeout_s)))
                                                     for c in cands], world, solves=3, warm=1, expect=expect,
                                                    sync=lambda: torch.cuda.synchronize(device), log=log)
        info = {c["name"]: c for c in cands}
        if sol is not None:
            sol.close()  # rebuilt below with the requested hand-off deadline (collective)
            sol = info[winner]["build"](timeout_s)
        tour_wall_s = time.perf_counter() - t_tour  # builds + untimed solves of every candidate + the rebuild
    if sol is None:
        halo = None
        if args.engine == "replicated-halo" and world > 1:
            from gadmm_amd.data import linear_synthetic
            ds_all = linear_synthetic(args.workers)  # opt-in: the halo engine needs other ranks' shards
            halo = (ds_all.X, ds_all.y)
        eng = "graph" if (tournament is not None) else args.engine  # nothing won: the graph engine
        sol = DistributedChainSolver(X_cpu.to(device).contiguous(), y_cpu.to(device).contiguous(), local,
                                     args.workers, placement, rank, world, device, args.rho, obj0, args.tol,
                                     engine=eng, fabric=args.fabric, share=share, block=args.block,
                                     halo_data=halo, use_graph=not args.no_graph, timeout_s=timeout_s)
    stall = os.environ.get("GADMM_BENCH_STALL", "")  # test hook "step:rank": that rank stalls before that step
    stall_step, stall_rank = (int(v) for v in stall.split(":")) if stall else (-1, -1)
    restarts = 0
    while True:
        for _ in range(args.warmup):
            if sol.solve_agreed().done != 1:  # collective: a failure anywhere moves every rank to the graph engine
                raise BenchFailure("a warm-up solve did not converge (fabric %s, fallbacks %s)"
                                   % (sol.kind, sol.fallbacks))
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        results, stamps = [], []
        t0 = time.perf_counter()
        for k in range(args.steps):
            if k == stall_step and rank == stall_rank and restarts == 0:
                sol.delay_next_s = 3.0 * timeout_s
            results.append(sol.guarded_solve())
            stamps.append(time.perf_counter())  # every solve ends in its own stream sync (per-step record)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        # every timed solve must have converged in the same (reference) iteration count, on every rank
        its = {r.iters for r in results}
        good = all(r.done == 1 for r in results) and len(its) == 1 and (expect is None or its == {expect})
        if good and world > 1:
            from gadmm_amd.engine.tournament import ranks_agree
            good = ranks_agree(next(iter(its)), world)
        if all_ok(good, world):
            break
        # collective fallback: every rank leaves the persistent engine for the graph engine together and
        # the timing restarts there (warm-up + K steps); the JSON line names the fallback
        if world == 1 or not sol.can_fall_back() or restarts >= 1:
            raise BenchFailure("timed solves: done=%s iterations=%s (expected %s)"
                               % (sorted({r.done for r in results}), sorted(its), expect))
        sol.fall_back("timed solve failed on some rank (done=%s here); timing restarted"
                      % sorted({r.done for r in results}))
        restarts += 1
    ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    if tournament is not None:
        # the tournament's cost model, predicted_ms = iters x (one-GPU us + hops x hop us), reported per
        # candidate next to its measured time. The compute term is rank 0's one-GPU blocked solve measured
        # on this box AFTER the timed solves (run before them, its leftover stream slowed the later
        # candidates of a 4-rank shared-GPU rehearsal by up to 11 %: profiles/r06_b/calib), the other
        # families scaled by the ONE_GPU_US ratios; model_error = measured / predicted - 1 (ranks
        # time-sharing one GPU inflate it: the model has no term for that)
        if os.environ.get("GADMM_TOURNAMENT_CALIBRATE", "1") != "0":
            calib_us = _one_gpu_calibration(args, rank, world, device, obj0)
        hop_us = max([h for h in (hop or {}).get("hop_us", []) if h is not None], default=None)
        scale = (calib_us / ONE_GPU_US["blocked"]) if calib_us else 1.0
        for row in tournament:
            c = info[row["engine"]]
            row["hops_per_iter"] = round(c["hops"], 4)
            its = row["iters"] if isinstance(row["iters"], int) else expect
            row["predicted_ms"] = (round(its * (scale * ONE_GPU_US[c["base"]] + c["hops"] * hop_us) / 1e3, 4)
                                   if (c["base"] and hop_us is not None and its) else None)
            row["model_error"] = (round(row["ms"] / row["predicted_ms"] - 1.0, 3)
                                  if row.get("predicted_ms") and row.get("ok") and row.get("ms") else None)
    last = results[-1]
    iters, p2p, wire, mon, repl = last.iters, last.theta_bytes, last.wire_bytes, last.monitor_bytes, sol.replicated_bytes
    if world > 1:
        t = torch.tensor([ms, float(p2p), float(wire), float(mon), float(repl)], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        ms = float(mx[0])
        p2p, wire, mon, repl = int(sm[1]), int(sm[2]), int(sm[3]), int(sm[4])
    tr = sol.objective_trace(iters)
    gap = abs(float(tr[iters - 1]) - obj0) if iters > 0 else float("nan")
    dl_mode = sol.blk is None or sol.blk.data_local  # theta-only exchange (payload formula below)
    data_local = dl_mode and repl == 0  # the halo mode also holds one neighbour head's shard per boundary
    per = np.diff(np.asarray([t0] + stamps)) * 1e3  # this rank's per-step wall times
    if rank == 0:
        value = ms / 1e3
        out = {
            "metric": "wall-clock to 1e-8 objective gap, GADMM linear regression (LinearRegression_Synthetic)",
            "value": round(value, 6),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": round(value / BASELINE_S, 6),
            "dtype": "fp64",
            "data": "synthetic (reference LinearRegression_Synthetic design rebuilt from shipped inputData.mat)",
            "config": {"model": "LinearRegression_Synthetic GADMM closed-form", "workers": args.workers,
                       "features": d, "samples_per_worker": m, "rho": args.rho,
                       "tol": args.tol, "global_batch": args.workers * m, "seq_len": 1,
                       "parallelism": "chain%d-over-%dgpu" % (args.workers, world)},
            "iterations_to_tol": iters,
            "expected_iterations": expect,
            "iterations_match_reference": (iters == expect) if expect else None,
            "final_gap": gap,
            "data_local": data_local,
            # theta over the fabric per solve, all ranks, iterations 1..iters: a data-local chain sends
            # 2 messages of d doubles per rank boundary per iteration (group_ADMM_closedForm.m:18-27, 62-70)
            "comm_bytes_per_solve": p2p,
            "theta_payload_bytes_per_solve": p2p,
            "theta_payload_bytes_formula": 2 * (world - 1) * d * 8 * iters if dl_mode else None,
            "wire_bytes_per_solve": wire,
            "monitor_bytes_per_solve": mon,
            "replicated_shard_bytes": repl,
            "p2p_messages_per_iteration": chain_message_count(list(range(args.workers)), placement),
            "us_per_iteration": round(ms * 1e3 / max(iters, 1), 3),
            "step_ms_min": round(float(np.min(per)), 4) if len(per) else None,
            "step_ms_median": round(float(np.median(per)), 4) if len(per) else None,
            "step_ms_max": round(float(np.max(per)), 4) if len(per) else None,
            "engine": sol.engine_name(),
            "kernel": sol.kernel,
            "fabric": sol.kind,
            "fallbacks": sol.fallbacks,
            "timing_restarts": restarts,
            "setup_in_timed_region": True,  # every step: Gram + b + y'y (f64 MFMA), inverses, iterations
            "baseline_s": BASELINE_S,
        }
        if hop is not None:
            out["xgmi_hop_us"] = hop.get("hop_us")  # one-way, per chain boundary (rank r -> r + 1)
            out["hop_probe_same_device"] = hop.get("same_device")  # ranks sharing one GPU (rehearsal)
        if tournament is not None:
            out["engine_tournament"] = tournament  # every candidate's untimed-warm-up time (max over ranks)
            out["tournament_winner"] = winner
            out["tournament_deadline_s"] = tour_timeout_s
            out["tournament_wall_s"] = round(tour_wall_s, 3)
            out["one_gpu_us_per_iter_measured"] = round(calib_us, 4) if calib_us else None
            out["rccl_built"] = any(row.get("engine") == "graph-rccl" for row in tournament)
        out["handoff_deadline_s"] = timeout_s  # the deadline of the warm-up and timed solves
        print(json.dumps(out), flush=True)
    sol.close()


def run_cpu_gloo(args, rank, world):
    """BASELINE.json configs[0]: LinearRegression_Synthetic closed-form GADMM with the workers spread
    over ``world`` CPU processes on gloo (torch path: batched local solves, neighbour theta by gloo
    isend/irecv), timed like the headline. A plumbing check of the distributed path, not a GPU
    number."""
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.benchmarks import headline_rank_problem, EXPECTED_ITERS_1E8
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.parallel.comm import LocalComm, TorchDistComm

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = TorchDistComm() if world > 1 else LocalComm()
    X, y, local, placement, obj0 = headline_rank_problem(args.workers, rank, world)
    m = LinearRegression(X, y)
    expect = EXPECTED_ITERS_1E8.get((args.workers, float(args.rho))) if args.tol == 1e-8 else None

    def solve():
        return chain_admm(m, local, args.workers, args.rho, obj0, args.tol, 20000, comm=comm, placement=placement,
                          backend="torch")

    for _ in range(args.warmup):
        solve()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    rs = [solve() for _ in range(args.steps)]
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    its = {r.iters for r in rs}
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    r = rs[-1]
    if rank == 0:
        print(json.dumps({
            "metric": "wall-clock to 1e-8 objective gap, GADMM linear regression (LinearRegression_Synthetic), "
                      "CPU gloo ranks (BASELINE configs[0] plumbing)",
            "value": round(ms / 1e3, 6), "unit": "s", "n_gpus": 0, "cpu_ranks": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": False, "scaling": "strong",
            "vs_baseline": round(ms / 1e3 / BASELINE_S, 6), "dtype": "fp64",
            "data": "synthetic (reference LinearRegression_Synthetic design rebuilt from shipped inputData.mat)",
            "config": {"model": "LinearRegression_Synthetic GADMM closed-form", "workers": args.workers,
                       "rho": args.rho, "tol": args.tol, "global_batch": args.workers * 50, "seq_len": 1,
                       "parallelism": "chain%d-over-%d-gloo-ranks" % (args.workers, world)},
            "iterations_to_tol": r.iters, "expected_iterations": expect,
            "iterations_match_reference": (its == {expect}) if expect else None,
            "theta_payload_bytes_per_solve": int(r.bytes_total), "backend": "torch+gloo"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_other(args, rank, world, device, share):
    from gadmm_amd.benchmarks import CONFIGS

    comm = None
    args.share = share
    if world == 1:
        from gadmm_amd.parallel.comm import LocalComm
        comm = LocalComm()
    # several ranks: no communicator up front -- a body that needs a data plane builds it lazily
    # (benchmarks.rank_comm: the IPC transport by default, RCCL with its watchdog for --fabric rccl)
    r = CONFIGS[args.config](args, rank, world, device, comm)
    if rank == 0:
        value = r["ms"] / 1e3
        out = {"metric": r["metric"], "value": round(value, 6), "unit": "s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(r["ms"], 4), "higher_is_better": False,
               "scaling": "weak" if args.config == "real10m" else "strong", "vs_baseline": None, "dtype": "fp64",
               "data": "synthetic (random-init / reference-shaped, generated on device)", "config": r["config"],
               "iterations_to_tol": r["iters"], "expected_iterations": r["expected"],
               "iterations_match_reference": (r["iters"] == r["expected"]) if r["expected"] else None,
               "backend": r.get("backend")}
        for k, v in r.items():
            if k not in out and k not in ("ms", "iters", "expected", "metric", "config"):
                out[k] = v
        from gadmm_amd.benchmarks import LAST_STEPS
        for k, v in LAST_STEPS.items():
            out.setdefault(k, v)
        print(json.dumps(out), flush=True)
    if comm is not None and hasattr(comm, "close"):
        comm.close()


if __name__ == "__main__":
    main()
