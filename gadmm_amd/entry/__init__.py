"""Entry points named after the reference scripts."""
ENTRIES = ["LinearRegression_Synthetic", "LinearRegression_Real", "LogisticRegression_Synthetic",
           "LogisticRegression_Real", "Dynamic_LinearRegression_Synthetic", "Dynamic_LinearRegression_Real",
           "LinearRegression_gadmm_vs_admm", "LinearRegression_RealShaped"]


def get(name: str):
    import importlib

    low = {e.lower(): e for e in ENTRIES}
    key = low.get(name.lower())
    if key is None:
        raise KeyError("unknown entry point %r; available: %s" % (name, ", ".join(ENTRIES)))
    return importlib.import_module("gadmm_amd.entry." + key)
