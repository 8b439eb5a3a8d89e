"""E6 — ``dynamic_LinearRegression_Real.m``: Body Fat (10 workers x 25 rows), rho = 0.1,
D-GADMM with coherence 50 (<= 20,000 iterations). The reference's second curve calls the missing
``dynamic_group_ADMM_closedForm_v2`` and is not reproducible; only the A4 run is."""
import numpy as np

from ..algorithms import dynamic_group_admm
from ..parallel import topology as T
from .common import Problem, run_entry

ENTRY = "Dynamic_LinearRegression_Real"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    rng = np.random.default_rng(cfg.path_seed)
    path, cost, _ = T.find_path(prob.n_total, rng)
    runs = {}
    for coh in cfg.coherences:
        r = dynamic_group_admm(prob.model, cfg.rhos[0], prob.obj0, cfg.acc, cfg.gadmm_iters, path, cost, coh,
                               seed=cfg.path_seed, n_total=prob.n_total, local_ids=prob.local_ids,
                               placement=prob.placement, backend=args.backend,
                               **sess.chain_kw(prob.n_total, prob.d, dynamic=float(coh) < cfg.gadmm_iters + 1))
        r.extra.pop("engine_obj", None)
        r.extra.pop("state", None)
        runs["D-GADMM(coh=%g)" % coh] = r
    return {"runs": runs, "obj0": prob.obj0, "dataset": prob.dataset_meta,
            "note": "dynamic_group_ADMM_closedForm_v2 is referenced but not shipped (SURVEY.md D8)",
            "figure_groups": {"Dynamic_LinearRegression_Real": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
