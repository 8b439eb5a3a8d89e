"""E4 — ``LogisticRegression_real.m``: Derm (data11) split over N = 10 workers
(``per_split = floor(n/N)``), lambda = 1e-5; baselines 100,000 iterations, dual averaging up to
500,000; GADMM with inexact local GD (step 0.08) for rho in {0.03, 0.02} (<= 1000 iterations).
``--set data_dir=/path/to/data11`` loads the UCI files; otherwise a 358 x 34 real-shaped synthetic
stand-in with +-1 labels is used."""
from .common import Problem, baselines, gadmm_sweep, maybe_checkpoint, run_entry

ENTRY = "LogisticRegression_Real"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    runs = {}
    b = baselines(prob, sess)
    obj0_gd = b.pop("_obj0_gd", None)
    runs.update(b)
    runs.update(gadmm_sweep(prob, sess, args.backend, state_rho=cfg.rhos[-1] if args.checkpoint else None))
    ck = maybe_checkpoint(args, sess, prob, runs["GADMM_rho%g" % cfg.rhos[-1]], cfg.rhos[-1], "GADMM-logistic")
    return {"runs": runs, "obj0": prob.obj0, "obj0_gd": obj0_gd, "checkpoint": ck, "dataset": prob.dataset_meta,
            "figure_groups": {"LogisticRegression_Real": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
