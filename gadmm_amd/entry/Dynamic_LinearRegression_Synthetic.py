"""E5 — ``Dynamic_LinearRegression_Synthetic.m``: N = 50 workers (E1 design), rho = 3, <= 5000
iterations.

Part 1 (:83-125): a fixed chain ``path0`` from ``findPath`` and ``n_pregen_paths`` pre-drawn node
geometries; the static-chain GADMM pays ``calc_cost(grid_k, path0)`` (A6) while D-GADMM v0 re-chains
to the k-th greedy path every 10 iterations (A5). D-GADMM's cost and clock are inflated by
x(1 + 5/15) for re-chaining overhead (:123,125).
Part 2 (:142-173): D-GADMM (A4, findPath2 re-chaining) for coherence in {1e9, 1, 10, 50, 100}.
All chains come from one seeded RNG, so every rank derives the same sequence with no message."""
import numpy as np

from ..algorithms import dynamic_group_admm, dynamic_group_admm_v0, static_group_admm
from ..parallel import topology as T
from .common import Problem, run_entry

ENTRY = "Dynamic_LinearRegression_Synthetic"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    N, rho = prob.n_total, cfg.rhos[0]
    rng = np.random.default_rng(cfg.path_seed)
    path0, cost0, grid = T.find_path(N, rng)
    paths, costs, static_costs = [path0], [cost0], [T.calc_cost(grid, path0)]
    for _ in range(cfg.n_pregen_paths):
        p, c, g = T.find_path(N, rng)
        paths.append(p)
        costs.append(c)
        static_costs.append(T.calc_cost(g, path0))
    costs = np.asarray(costs)
    static_costs = np.asarray(static_costs)
    kw = dict(n_total=N, local_ids=prob.local_ids, placement=prob.placement, backend=args.backend)

    def fab(coh):  # several GPUs: the persistent kernels over xGMI (D-GADMM: a ring of table slots)
        return sess.chain_kw(N, prob.d, dynamic=float(coh) < cfg.gadmm_iters + 1)

    runs = {}
    # the identity chain is the static GADMM of A6 (path0 only enters through the costs)
    runs["GADMM_static(coh=%g)" % cfg.coherence_v0] = static_group_admm(
        prob.model, rho, prob.obj0, cfg.acc, cfg.gadmm_iters, cfg.coherence_v0, static_costs, **kw,
        **fab(cfg.coherence_v0))
    r0 = dynamic_group_admm_v0(prob.model, rho, prob.obj0, cfg.acc, cfg.gadmm_iters, paths, costs,
                               cfg.coherence_v0, **kw, **fab(cfg.coherence_v0))
    infl = 1.0 + cfg.overhead_inflation
    r0.com_cost = r0.com_cost * infl
    r0.time_trace = r0.time_trace * infl
    r0.extra["inflation"] = infl
    runs["D-GADMM_v0(coh=%g)" % cfg.coherence_v0] = r0
    p1, c1, _ = T.find_path(N, rng)
    for coh in cfg.coherences:
        r = dynamic_group_admm(prob.model, rho, prob.obj0, cfg.acc, cfg.gadmm_iters, p1, c1, coh,
                               seed=cfg.path_seed + int(min(coh, 1e6)), **kw, **fab(coh))
        runs["D-GADMM(coh=%g)" % coh] = r
    for r in runs.values():
        r.extra.pop("engine_obj", None)
        r.extra.pop("state", None)
        if r.com_cost is not None and len(r.com_cost) == len(r.loss):
            r.comm_units = r.com_cost  # energy-cost axis, as the reference plots it
            r.extra["energy_units"] = True
    return {"runs": runs, "obj0": prob.obj0, "dataset": prob.dataset_meta,
            "figure_groups": {"D-GADMM vs static GADMM (N=%d)" % N: runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
