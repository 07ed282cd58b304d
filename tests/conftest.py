import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
for p in (str(REPO), str(REPO / "tests"), str(REPO / "k-step_fm-index_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def kfmi_mod():
    import kstep_fmi
    kstep_fmi.load()
    return kstep_fmi


def pytest_collection_modifyitems(config, items):
    # OMP inside the oracle: keep CPU tests bounded on small boxes.
    os.environ.setdefault("OMP_NUM_THREADS", "8")
