"""E3 — ``LogisticRegression_Synthetic.m``: N = 24, X_n = q_n q_n^T + I with +-1 labels (== the
shipped inputData.mat), lambda = 1e-5, Hmax_n = 1/4 lambda_max + lambda; baselines 100,000
iterations (the reference's optimum is the final GD objective — reported as ``obj0_gd`` next to the
certified Newton optimum used here); dual averaging; GADMM with inexact local GD (step 2.2) for
rho in {3e-4, 2e-4} (<= 400 iterations)."""
from .common import Problem, baselines, gadmm_sweep, maybe_checkpoint, run_entry

ENTRY = "LogisticRegression_Synthetic"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    sess.log("  obj0 = %.13f (Newton, N*lambda ridge)" % prob.obj0)
    runs = {}
    b = baselines(prob, sess)
    obj0_gd = b.pop("_obj0_gd", None)
    runs.update(b)
    runs.update(gadmm_sweep(prob, sess, args.backend, state_rho=cfg.rhos[-1] if args.checkpoint else None))
    ck = maybe_checkpoint(args, sess, prob, runs["GADMM_rho%g" % cfg.rhos[-1]], cfg.rhos[-1], "GADMM-logistic")
    return {"runs": runs, "obj0": prob.obj0, "obj0_gd": obj0_gd, "checkpoint": ck, "dataset": prob.dataset_meta,
            "figure_groups": {"LogisticRegression_Synthetic": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
