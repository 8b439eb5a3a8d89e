"""Summarise a rocprofv3 PMC database (``-o NAME`` -> NAME_results.db): per kernel (name matched by a
substring), the sum of every collected counter over its dispatches, plus derived stall fractions.

    python tools/pmc_summary.py gpurun_out/r5h2/pmc/pmc_results.db oz_gemm gram_aug
"""
import sqlite3
import sys
from collections import defaultdict


def summarise(db, patterns):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, dispatch_id, counter_name, value, duration from counters_collection")
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for name, did, cn, v, du in rows:
        for p in patterns:
            if p in name:
                acc[p][cn] += v
                disp[p].add(did)
                dur[p][did] = du
    out = []
    for p in patterns:
        if p not in acc:
            out.append("%s: no dispatches" % p)
            continue
        a = acc[p]
        out.append("%s: %d dispatches, %.3f ms total" % (p, len(disp[p]), sum(dur[p].values()) / 1e6))
        for k in sorted(a):
            out.append("  %-28s %.4g" % (k, a[k]))
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in a:
                    out.append("  %-28s %.1f %% of wave cycles" % (k, 100.0 * a[k] / wc))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "SQ_BUSY_CYCLES" in a:
            out.append("  MFMA busy / (SQ busy x CUs per SE x 4 SIMDs): see README (per-SE aggregation)")
    return "\n".join(out)


if __name__ == "__main__":
    print(summarise(sys.argv[1], sys.argv[2:]))
