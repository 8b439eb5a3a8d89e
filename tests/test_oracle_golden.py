"""The reference-semantics oracle reproduces the [measured-here] numbers of BASELINE.md."""
import numpy as np
import pytest

from gadmm_amd.oracle import reference as R


def test_linear_optimum(lin_obj0):
    assert lin_obj0 == pytest.approx(218.6486436261889, rel=1e-13)


def test_logistic_optimum(log_obj0):
    assert log_obj0 == pytest.approx(0.7177269844827, abs=1e-12)


@pytest.mark.parametrize("rho,it4,it8", [(7, 248, 428), (5, 434, 758)])
def test_gadmm_linear_iterations(lin24, lin_obj0, rho, it4, it8):
    X, y = lin24.numpy()
    r = R.gadmm_linear(X, y, rho, 3000, lin_obj0, 1e-8)
    assert r.iters == it8
    assert int(np.argmax(np.array(r.loss) < 1e-4)) + 1 == it4


def test_std_admm_iterations(lin24, lin_obj0):
    X, y = lin24.numpy()
    assert R.std_admm_linear(X, y, 1.0, 1000, lin_obj0, 1e-4).iters == 348


def test_dgadmm_identity_equals_gadmm(lin24, lin_obj0):
    X, y = lin24.numpy()
    a = R.gadmm_linear(X, y, 7, 600, lin_obj0, 1e-4)
    b = R.dgadmm_linear(X, y, 7, 600, lin_obj0, 1e-4, list(range(24)), np.zeros(23), 1e9)
    assert a.iters == b.iters == 248
    assert np.allclose(a.obj, b.obj, rtol=1e-12)


def test_logistic_gadmm_iterations(log24, log_obj0):
    X, y = log24.numpy()
    r = R.gadmm_logistic_gd(X, y, 2e-4, 100, log_obj0, 1e-5, 1e-4, 2.2)
    assert r.iters == 53
