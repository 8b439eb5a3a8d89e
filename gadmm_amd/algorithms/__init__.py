"""Distributed algorithms of the reference, on the MI355X fabric."""
from .base import RunResult, Stopper
from .gadmm import (chain_admm, group_admm_closed_form, group_admm_logistic_gd, group_admm_logistic_exact,
                    dynamic_group_admm, dynamic_group_admm_v0, static_group_admm)
from .std_admm import standard_admm
from .dual_averaging import dual_averaging
from .baselines import (gradient_descent, decentralized_gd, lag, iag, gd_dgd_lag, global_constants)

__all__ = ["RunResult", "Stopper", "chain_admm", "group_admm_closed_form", "group_admm_logistic_gd",
           "group_admm_logistic_exact", "dynamic_group_admm", "dynamic_group_admm_v0", "static_group_admm",
           "standard_admm", "dual_averaging", "gradient_descent", "decentralized_gd", "lag", "iag", "gd_dgd_lag",
           "global_constants"]
