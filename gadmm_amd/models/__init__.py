"""Model families: the reference's two consensus problems."""
from .linear import LinearRegression
from .logistic import LogisticRegression

MODELS = {"linear": LinearRegression, "logistic": LogisticRegression}


def make_model(kind: str, X, y, lam: float = 0.0):
    if kind == "linear":
        return LinearRegression(X, y, lam=lam)
    if kind == "logistic":
        return LogisticRegression(X, y, lam=lam)
    raise ValueError("unknown model kind %r" % kind)


__all__ = ["LinearRegression", "LogisticRegression", "MODELS", "make_model"]
