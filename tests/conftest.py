import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(autouse=True)
def _reset_mesh():
    from scaletorch_amd.parallel import mesh

    mesh.reset_process_group_manager()
    yield
    mesh.reset_process_group_manager()
