"""In-kernel timeline of the data-local multi-GPU chain kernel (chain_blocked.hip, blk_dl = 1) with
two ranks sharing cuda:0: where a boundary hand-off's time goes. Rank 1's wave 0 is its boundary head
(position 12), rank 0's tail wave 11 (dbg = 5 << 4) its boundary tail (position 11); s_memrealtime is
one clock for the chip, so push -> poll-success across ranks is a hop.

    python tools/dl_timeline.py [iters=200]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, K):
    import numpy as np
    import torch
    from gadmm_amd.benchmarks import headline_rank_problem
    from gadmm_amd.engine.blocked_xgmi import BlockedXgmiEngine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y, loc, pl, obj0 = headline_rank_problem(24, rank, world)
    eng = BlockedXgmiEngine(X, y, 24, pl, rank, 3.0, obj0, 1e-8, 3000, dev, data_local=True)
    for _ in range(2):
        eng.run()
    iters, done, ms = eng.run(timeline_iters=K, dbg=5 << 4)
    tl = eng.last_timeline
    eng.close()
    return {"iters": iters, "done": done, "ms": ms, "w0": tl[0].tolist(), "tail": tl[128].tolist()}


def main():
    import numpy as np
    from gadmm_amd.parallel.launch import spawn
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    os.environ.setdefault("GADMM_BENCH_SHARE_GPU", "1")
    res = spawn(_rank, 2, K, timeout=300)
    r0, r1 = res
    h = np.asarray(r1["w0"], dtype=np.float64)    # rank 1 wave 0 = boundary head (position 12)
    t = np.asarray(r0["tail"], dtype=np.float64)  # rank 0 tail wave 11 = boundary tail (position 11)
    ok = slice(5, K - 1)
    us = lambda v: float(np.median(v)) / 100.0
    out = {
        "iters": [r0["iters"], r1["iters"]], "ms": [r0["ms"], r1["ms"]],
        "rank1_head_period_us": us(np.diff(h[:, 0])[ok]),
        "rank1_head_poll_wait_us": us((h[:, 6] - h[:, 0])[ok]),      # iteration start -> its head solve starts
        "rank1_head_solve_us": us((h[:, 7] - h[:, 6])[ok]),
        "rank0_tail_poll_wait_us": us((t[:, 1] - t[:, 0])[ok]),     # tail phase start -> remote theta arrived
        "rank0_tail_solve_us": us((t[:, 2] - t[:, 1])[ok]),
        "rank0_tail_stores_us": us((t[:, 3] - t[:, 2])[ok]),
        # hop head -> tail: rank 1's push (right after its solve) to rank 0's poll success, same iteration
        "hop_head_to_tail_us": us((t[:, 1] - h[:, 7])[ok]),
        # hop tail -> head: rank 0's tail push (after its solve) to rank 1's next head solve start
        "hop_tail_to_head_us": us((h[1:, 6] - t[:-1, 2])[5:K - 2]),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
