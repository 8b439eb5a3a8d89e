"""Structured run outputs (SURVEY.md §5 Metrics/logging): per-iteration JSONL/CSV traces with the
objective, gap, reference communication units, real bytes and wall time, plus summaries and the
paper-style 3-panel figures (gap vs iteration / communication / clock)."""
from __future__ import annotations

import csv
import json
import os
from typing import Dict, Iterable, List, Optional

import numpy as np


def _clean(v):
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


class RunWriter:
    """Writes ``<outdir>/<name>.jsonl`` (one line per iteration), ``<name>.csv`` and appends to
    ``summary.json``. Only rank 0 writes."""

    def __init__(self, outdir: Optional[str], rank: int = 0):
        self.outdir = outdir
        self.rank = rank
        self.summary: Dict[str, Dict] = {}
        if outdir and rank == 0:
            os.makedirs(outdir, exist_ok=True)

    def add(self, key: str, result, every: int = 1, **extra) -> None:
        s = dict(result.summary())
        s.update({k: _clean(v) for k, v in extra.items()})
        self.summary[key] = s
        if not self.outdir or self.rank != 0:
            return
        n = len(result.obj)
        idx = range(0, n, max(1, every))
        rows = []
        for i in idx:
            row = {"iter": i + 1, "obj": float(result.obj[i]), "gap": float(result.loss[i])}
            if len(result.comm_units) > i:
                row["comm_units"] = float(result.comm_units[i])
            if len(result.time_trace) > i:
                row["wall_s"] = float(result.time_trace[i])
            mt = getattr(result, "model_time", None)
            if mt is not None and len(mt) > i:
                row["model_clock_s"] = float(mt[i])
            if result.com_cost is not None and len(result.com_cost) > i:
                row["com_cost"] = float(result.com_cost[i])
            pr = getattr(result, "primal_res", None)
            if pr is not None and len(pr) > i:
                row["primal_res"] = float(pr[i])
            rows.append(row)
        base = os.path.join(self.outdir, _safe(key))
        with open(base + ".jsonl", "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
        if rows:
            with open(base + ".csv", "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)

    def close(self, extra: Optional[Dict] = None) -> Optional[str]:
        if not self.outdir or self.rank != 0:
            return None
        out = {"runs": self.summary}
        if extra:
            out.update({k: _clean(v) for k, v in extra.items()})
        p = os.path.join(self.outdir, "summary.json")
        with open(p, "w") as f:
            json.dump(out, f, indent=1, default=_clean)
        return p


def _safe(key: str) -> str:
    return "".join(c if c.isalnum() or c in "-_." else "_" for c in key)


def plot_three_panel(results: Dict[str, object], path: str, title: str = "", xmax_iter: Optional[int] = None) -> bool:
    """Gap vs iteration, vs cumulative communication units, vs measured wall clock (the reference's
    semilogy figures, e.g. LinearRegression_Synthetic.m:146-248), plus a fourth panel with the
    reference's modelled ``2 * toc`` clock when any run carries one (``RunResult.model_time``).
    Returns False if matplotlib is unavailable."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover
        return False
    modelled = any(getattr(r, "model_time", None) is not None for r in results.values())
    fig, ax = plt.subplots(1, 4 if modelled else 3, figsize=(20 if modelled else 15, 4.2))
    for name, r in results.items():
        loss = np.maximum(np.asarray(r.loss), 1e-16)
        it = np.arange(1, len(loss) + 1)
        ax[0].semilogy(it, loss, label=name)
        if len(r.comm_units) == len(loss):
            ax[1].semilogy(r.comm_units, loss, label=name)
        if len(r.time_trace) == len(loss):
            ax[2].semilogy(r.time_trace, loss, label=name)
        mt = getattr(r, "model_time", None)
        if modelled and mt is not None and len(mt) == len(loss):
            ax[3].semilogy(mt, loss, label=name)
    ax[0].set_xlabel("iteration")
    ax[1].set_xlabel("cumulative communication (reference units)")
    ax[2].set_xlabel("wall clock, measured [s]")
    if modelled:
        ax[3].set_xlabel("modelled clock: 2 x local-solve time per iteration [s]")
    for a in ax:
        a.set_ylabel("|obj - obj*|")
        a.grid(True, which="both", alpha=0.3)
    if xmax_iter:
        ax[0].set_xlim(1, xmax_iter)
    ax[0].legend(fontsize=7)
    if title:
        fig.suptitle(title)
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)
    return True
