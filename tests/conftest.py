"""Shared pytest configuration.

Tests that need an MI355X are marked ``@pytest.mark.gpu``; everything else runs on CPU
(``pytest -m "not gpu"``), including multi-process paths over the gloo backend.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))   # test helpers (fake_pymongo)
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def _share_cpus_between_xdist_workers():
    """Under pytest-xdist every worker would run torch's CPU kernels on all cores: 5 workers x 8
    threads on 8 cores starved the long CPU tests (ASHA-vs-random quality, resume) past their
    timeouts.  Each worker gets its share of the cores; serial runs are unchanged."""
    n = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
    if not n:
        return
    share = max(1, (os.cpu_count() or 1) // max(1, int(n)))
    os.environ.setdefault("OMP_NUM_THREADS", str(share))
    try:
        import torch
        torch.set_num_threads(share)
    except Exception:  # pragma: no cover
        pass


def pytest_configure(config):
    _share_cpus_between_xdist_workers()
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X, gfx950) and the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
