import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # under pytest-xdist every worker would start a full-width torch thread pool: the tiny (50 x 50)
    # CPU ops then thrash 8 cores (a 14 s test took 30 min at -n 6); give each worker its share
    n_workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1"))
    if n_workers > 1:
        import torch

        torch.set_num_threads(max(1, (os.cpu_count() or 8) // n_workers))
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU run (reference-length baselines)")


def pytest_collection_modifyitems(config, items):
    import torch

    has_gpu = torch.cuda.is_available()
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords and not has_gpu:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def lin24():
    from gadmm_amd.data import linear_synthetic

    return linear_synthetic(24)


@pytest.fixture(scope="session")
def log24():
    from gadmm_amd.data import logistic_synthetic

    return logistic_synthetic(24)


@pytest.fixture(scope="session")
def lin_obj0(lin24):
    from gadmm_amd.oracle.reference import opt_linear

    Xf, yf = lin24.stacked()
    return opt_linear(Xf.numpy(), yf.numpy())


@pytest.fixture(scope="session")
def log_obj0(log24):
    from gadmm_amd.oracle.reference import logistic_optimum

    Xf, yf = log24.stacked()
    return logistic_optimum(Xf.numpy(), yf.numpy(), 24 * 1e-5)
