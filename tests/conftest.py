import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def backend():
    from low_level_feature_extraction_amd.backend import Backend

    return Backend.get(0)


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle

    oracle.lib()
    return oracle


def pytest_sessionfinish(session, exitstatus):
    """Write the observed k-means parity statistics (tests/kmeans_bar.py) of a GPU run."""
    try:
        from tests import kmeans_bar
    except ImportError:  # pragma: no cover
        return
    summ = kmeans_bar.summary()
    if summ:
        import json

        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "kmeans_parity_observed.json"), "w") as f:
            json.dump(summ, f, indent=1)
