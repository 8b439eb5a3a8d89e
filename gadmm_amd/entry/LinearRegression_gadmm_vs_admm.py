"""E7 — ``LinearRegression_gadmm_vs_admm.m``: E1 data (N = 24), rho = 1, <= 20,000 iterations:
standard star ADMM (hub = worker N, reduce + broadcast on the fabric), GADMM, and D-GADMM with
coherence in {1, 10, 50}. Energy accounting from ``findPath2`` (:82-87): star cost per iteration =
sum(P_central) + max(P_central), chain cost = sum(pathCost) of the *initial* chain for every GADMM
variant (:128-179; the quirk that ignores D-GADMM's own com_cost is kept)."""
import numpy as np

from ..algorithms import dynamic_group_admm, standard_admm
from ..parallel import topology as T
from .common import Problem, gadmm_solve, run_entry

ENTRY = "LinearRegression_gadmm_vs_admm"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    rho = cfg.rhos[0]
    rng = np.random.default_rng(cfg.path_seed)
    path, cost, grid, p_central, center = T.find_path2(prob.n_total, rng)
    star = T.star_cost(p_central)
    chain = float(np.sum(cost))
    runs = {}
    # several GPUs: each comparator on its persistent kernel (star hub fan-in / the data-local chain /
    # D-GADMM's re-chaining kernel) over xGMI, the IPC transport as data plane (parallel/node.py)
    r = standard_admm(prob.model, prob.local_ids, prob.n_total, rho, prob.obj0, cfg.acc, cfg.gadmm_iters,
                      placement=prob.placement, backend=args.backend, **sess.star_kw(prob.n_total, prob.d))
    r.com_cost = np.arange(1, len(r.loss) + 1) * star
    runs["ADMM(star)"] = r
    g = gadmm_solve(prob, sess, rho, cfg.acc, cfg.gadmm_iters, args.backend, name="GADMM")
    runs["GADMM"] = g
    for coh in cfg.coherences:
        runs["D-GADMM(coh=%g)" % coh] = dynamic_group_admm(
            prob.model, rho, prob.obj0, cfg.acc, cfg.gadmm_iters, path, cost, coh, seed=cfg.path_seed + int(coh),
            n_total=prob.n_total, local_ids=prob.local_ids, placement=prob.placement, backend=args.backend,
            **sess.chain_kw(prob.n_total, prob.d, dynamic=float(coh) < cfg.gadmm_iters + 1))
    for k, v in runs.items():
        v.extra.pop("engine_obj", None)
        v.extra.pop("state", None)
        if k != "ADMM(star)":
            v.com_cost = np.arange(1, len(v.loss) + 1) * chain
        v.comm_units = v.com_cost
        v.extra["energy_units"] = True
    return {"runs": runs, "obj0": prob.obj0, "star_energy_per_iter": star, "chain_energy_per_iter": chain,
            "center": int(center), "dataset": prob.dataset_meta,
            "figure_groups": {"GADMM vs star ADMM (energy)": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
