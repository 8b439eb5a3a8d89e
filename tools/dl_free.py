"""Is the data-local multi-rank chain paced by its hand-offs or by its stop-rule pipeline? Two ranks
share cuda:0 and run the instrumented data-local kernel (chain_blocked.hip, TL build) twice:
dbg = 0 (normal: objective waves -> rank 0's monitor -> decision rings, workers poll the decision
LAG iterations behind) and dbg = 3 (experiment bits: the workers neither post objective values nor
poll decisions, so they run free to max_iter while the hand-offs between the ranks stay). The
iteration period of rank 1's wave 0 (its boundary head) comes from its s_memrealtime stamps; the
free run ends by a deadline (done = 4), which this tool expects.

    python tools/dl_free.py [iters=300]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, K):
    import torch
    from gadmm_amd.benchmarks import headline_rank_problem
    from gadmm_amd.engine.blocked_xgmi import BlockedXgmiEngine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y, loc, pl, obj0 = headline_rank_problem(24, rank, world)
    eng = BlockedXgmiEngine(X, y, 24, pl, rank, 3.0, obj0, 1e-8, 3000, dev, data_local=True)
    eng.run()
    out = {}
    for name, dbg, tmo in (("normal", 0, 20.0), ("free", 3, 0.5)):
        os.environ["GADMM_BLK_DBG"] = str(dbg | (5 << 4))  # the launcher takes the bits from here
        try:
            iters, done, ms = eng.run(timeline_iters=K, dbg=dbg | (5 << 4), timeout_s=tmo)
        except RuntimeError:
            iters, done, ms = -1, 4, -1.0
        out[name] = {"iters": iters, "done": done, "ms": ms, "w0": eng.last_timeline[0].tolist()}
    eng.close()
    return out


def main():
    import numpy as np
    from gadmm_amd.parallel.launch import spawn
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    os.environ.setdefault("GADMM_BENCH_SHARE_GPU", "1")
    res = spawn(_rank, 2, K, timeout=300)
    out = {}
    for name in ("normal", "free"):
        h = np.asarray(res[1][name]["w0"], dtype=np.float64)
        out[name + "_period_us"] = float(np.median(np.diff(h[:, 0])[5:K - 1])) / 100.0
        out[name + "_iters"] = res[0][name]["iters"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
