"""pytest configuration: the ``gpu`` marker (tests that need an MI355X; the CPU suite runs
``-m "not gpu"``) and the repository root on ``sys.path``."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running simulation test")


@pytest.fixture(autouse=True)
def _reset_known_geometries():
    from walkai_nos_amd.models.xcp import known_configs
    known_configs.reset_known_geometries()
    yield
    known_configs.reset_known_geometries()
