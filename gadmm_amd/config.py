"""Named experiment presets — one per reference entry script, defaults = the
reference's hard-coded values. Every field can be overridden from the CLI
(``python -m gadmm_amd <Entry> --set key=value``).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class ExperimentConfig:
    name: str
    model: str                      # 'linear' | 'logistic'
    data: str                       # 'linear_synthetic' | 'logistic_synthetic' | 'bodyfat' | 'derm' | 'gaussian'
    num_workers: int = 24
    rows_per_worker: int = 50       # real-shaped data: rows per worker (per_split)
    dim: int = 50
    total_rows: int = 0             # real-shaped data: dataset height before splitting
    baseline_iters: int = 60000
    dualavg_iters: Optional[int] = None
    gadmm_iters: int = 1000
    rhos: List[float] = field(default_factory=lambda: [3.0, 5.0, 7.0])
    acc: float = 1e-4
    lam: float = 0.0
    gd_step: float = 2.2            # logistic inner GD step (gdStep)
    max_inner: int = 100
    coherences: List[float] = field(default_factory=list)
    # logistic: extra GADMM runs with EXACT local solves (group_ADMM_logistic.m / SURVEY.md D2, the
    # Newton HIP kernel), which reach gaps the linearised inner GD cannot (SURVEY.md §7.3 "report both")
    exact_rhos: List[float] = field(default_factory=list)
    exact_acc: float = 1e-8
    exact_iters: int = 2000
    coherence_v0: float = 10.0
    n_pregen_paths: int = 1000
    overhead_inflation: float = 5.0 / 15.0   # Dynamic_LinearRegression_Synthetic.m:123,125
    run_baselines: bool = True
    run_dualavg: bool = True
    run_star: bool = False
    seed: int = 0
    path_seed: int = 1234
    data_dir: Optional[str] = None  # directory with data.txt / y.txt (reference UCI layout)
    reference: str = ""             # reference script this preset mirrors

    def override(self, **kw) -> "ExperimentConfig":
        return dataclasses.replace(self, **kw)

    def quick(self) -> "ExperimentConfig":
        """Reduced budgets for smoke tests (same structure, fewer iterations)."""
        return self.override(baseline_iters=min(self.baseline_iters, 300),
                             dualavg_iters=min(self.dualavg_iters or self.baseline_iters, 300),
                             gadmm_iters=min(self.gadmm_iters, 400), n_pregen_paths=min(self.n_pregen_paths, 60),
                             exact_iters=min(self.exact_iters, 60))


PRESETS = {
    "LinearRegression_Synthetic": ExperimentConfig(
        name="LinearRegression_Synthetic", model="linear", data="linear_synthetic", num_workers=24,
        baseline_iters=60000, gadmm_iters=1000, rhos=[3.0, 5.0, 7.0], acc=1e-4,
        reference="LinearRegression_Synthetic.m:14-17,78-94"),
    "LinearRegression_Real": ExperimentConfig(
        name="LinearRegression_Real", model="linear", data="bodyfat", rows_per_worker=25, dim=14,
        total_rows=252, num_workers=10, baseline_iters=40000, gadmm_iters=800, rhos=[3.0, 5.0, 7.0], acc=1e-4,
        reference="LinearRegression_Real.m:13-18,84-98"),
    "LogisticRegression_Synthetic": ExperimentConfig(
        name="LogisticRegression_Synthetic", model="logistic", data="logistic_synthetic", num_workers=24,
        baseline_iters=100000, gadmm_iters=400, rhos=[3e-4, 2e-4], acc=1e-4, lam=1e-5, gd_step=2.2,
        exact_rhos=[1e-3], reference="LogisticRegression_Synthetic.m:14-17,40-46,88-100"),
    "LogisticRegression_Real": ExperimentConfig(
        name="LogisticRegression_Real", model="logistic", data="derm", num_workers=10, dim=34, total_rows=358,
        baseline_iters=100000, dualavg_iters=500000, gadmm_iters=1000, rhos=[0.03, 0.02], acc=1e-4, lam=1e-5,
        gd_step=0.08, exact_rhos=[0.02], reference="LogisticRegression_real.m:17-34,46-47,65-85"),
    "Dynamic_LinearRegression_Synthetic": ExperimentConfig(
        name="Dynamic_LinearRegression_Synthetic", model="linear", data="linear_synthetic", num_workers=50,
        gadmm_iters=5000, rhos=[3.0], acc=1e-4, coherences=[1e9, 1, 10, 50, 100], coherence_v0=10,
        n_pregen_paths=1000, run_baselines=False, run_dualavg=False,
        reference="Dynamic_LinearRegression_Synthetic.m:17-37,78-173"),
    "Dynamic_LinearRegression_Real": ExperimentConfig(
        name="Dynamic_LinearRegression_Real", model="linear", data="bodyfat", rows_per_worker=25, dim=14,
        total_rows=252, num_workers=10, gadmm_iters=20000, rhos=[0.1], acc=1e-4, coherences=[50],
        run_baselines=False, run_dualavg=False, reference="dynamic_LinearRegression_Real.m:13-18,84-101"),
    "LinearRegression_gadmm_vs_admm": ExperimentConfig(
        name="LinearRegression_gadmm_vs_admm", model="linear", data="linear_synthetic", num_workers=24,
        gadmm_iters=20000, rhos=[1.0], acc=1e-4, coherences=[1, 10, 50], run_baselines=False, run_dualavg=False,
        run_star=True, reference="LinearRegression_gadmm_vs_admm.m:78-119"),
}


def get_preset(name: str) -> ExperimentConfig:
    if name.lower() == "linearregression_realshaped":
        from .entry import LinearRegression_RealShaped  # noqa: F401  (registers its preset)
    key = {k.lower(): k for k in PRESETS}.get(name.lower())
    if key is None:
        raise KeyError("unknown entry point %r (have: %s)" % (name, ", ".join(PRESETS)))
    return PRESETS[key]


def parse_overrides(cfg: ExperimentConfig, items: List[str]) -> ExperimentConfig:
    """``key=value`` overrides; lists as comma-separated values."""
    kw = {}
    fields = {f.name: f for f in dataclasses.fields(cfg)}
    for it in items or []:
        k, v = it.split("=", 1)
        if k not in fields:
            raise KeyError("unknown config field %r" % k)
        cur = getattr(cfg, k)
        if isinstance(cur, bool):
            kw[k] = v.lower() in ("1", "true", "yes")
        elif isinstance(cur, int) and not isinstance(cur, bool):
            kw[k] = int(float(v))
        elif isinstance(cur, float):
            kw[k] = float(v)
        elif isinstance(cur, list):
            kw[k] = [float(x) for x in v.split(",") if x]
        elif cur is None and k == "dualavg_iters":
            kw[k] = int(float(v))
        else:
            kw[k] = v
    return cfg.override(**kw)
