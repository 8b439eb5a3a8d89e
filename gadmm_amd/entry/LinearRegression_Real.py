"""E2 — ``LinearRegression_Real.m``: Body Fat (data29) split into ``floor(252/25) = 10`` workers of
25 rows; baselines 40,000 iterations; GADMM rho in {3, 5, 7} (<= 800 iterations).
The UCI file is not shipped with the reference: ``--set data_dir=/path/to/data29`` loads it
(``data.txt``/``y.txt``), otherwise a real-*shaped* synthetic stand-in (252 x 14) is used."""
from .common import Problem, baselines, gadmm_sweep, maybe_checkpoint, run_entry

ENTRY = "LinearRegression_Real"


def body(cfg, sess, args, writer):
    prob = Problem(cfg, sess)
    runs = {}
    runs.update(baselines(prob, sess))
    runs.pop("_obj0_gd", None)
    runs.update(gadmm_sweep(prob, sess, args.backend, state_rho=cfg.rhos[-1] if args.checkpoint else None))
    ck = maybe_checkpoint(args, sess, prob, runs["GADMM_rho%g" % cfg.rhos[-1]], cfg.rhos[-1], "GADMM")
    return {"runs": runs, "obj0": prob.obj0, "checkpoint": ck, "dataset": prob.dataset_meta,
            "figure_groups": {"LinearRegression_Real": runs}}


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
