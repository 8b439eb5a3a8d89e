"""E1 — ``LinearRegression_Synthetic.m``: N = 24 workers, X_n = 1.3^(n-1) q_n q_n^T + I (50 x 50),
baselines GD/DGD/LAG-PS/LAG-WK/cIAG/R-IAG (60,000 iterations) and dual averaging, then GADMM with
rho in {3, 5, 7} (<= 1000 iterations, acc = 1e-4). Outputs the reference's three panels (gap vs
iteration / cumulative communication / clock) and per-run traces."""
from .common import Problem, baselines, gadmm_sweep, maybe_checkpoint, run_entry

ENTRY = "LinearRegression_Synthetic"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    sess.log("  obj0 = %.13f (normal equations, opt_sol_closedForm.m)" % prob.obj0)
    runs = {}
    runs.update(baselines(prob, sess))
    runs.pop("_obj0_gd", None)
    runs.update(gadmm_sweep(prob, sess, args.backend, state_rho=cfg.rhos[-1] if args.checkpoint else None))
    last = runs["GADMM_rho%g" % cfg.rhos[-1]]
    ck = maybe_checkpoint(args, sess, prob, last, cfg.rhos[-1], "GADMM")
    return {"runs": runs, "obj0": prob.obj0, "checkpoint": ck, "dataset": prob.dataset_meta,
            "figure_groups": {"LinearRegression_Synthetic": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
