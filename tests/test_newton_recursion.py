"""Host check of the algebra behind the exact-logistic pipeline kernel (chain_persistent_newton.hip,
chain_persistent_newton_rec_kernel): the chord-Newton step with the margins carried by the recursion
z_{k+1} = z_k - X P y_k + X P X^T s_k (tools/newton_recursion_emul.py, f64 numpy) reaches the 1e-8 gap
of the bench config logistic_exact in the reference's 424 iterations, with the same chord steps and
theta within 1e-12 of the direct step x' = x - P g(x)."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _emul():
    spec = importlib.util.spec_from_file_location("newton_recursion_emul",
                                                  os.path.join(ROOT, "tools", "newton_recursion_emul.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_margins_recursion_keeps_reference_iterations():
    emul = _emul()
    it_d, st_d, th_d = emul.run("direct")
    it_r, st_r, th_r = emul.run("rec")
    assert it_d == it_r == 424
    assert np.array_equal(st_d, st_r)
    assert np.abs(th_r - th_d).max() <= 1e-12 * np.abs(th_d).max()
