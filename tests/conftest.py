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


#: GPU tests that measure how pod PROCESSES share the GPU run before every test that opens streams
#: in this pytest process: the kernel tests leave this process's CU-masked streams (hardware queues)
#: on the GPU, a node's agents hold none (they never open a GPU context), and queues of a process
#: that is not a pod perturb how the hardware deals the pods' queues over its pipes
#: (profiles/churn_probe_r6.json). The order within each group is kept.
_PROCESS_SHARING = ("share_compute_evenly", "share_one_gpu_evenly")


def pytest_collection_modifyitems(session, config, items):
    first = [it for it in items if any(k in it.nodeid for k in _PROCESS_SHARING)]
    if first:
        rest = [it for it in items if not any(k in it.nodeid for k in _PROCESS_SHARING)]
        items[:] = first + rest
