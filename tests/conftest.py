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


@pytest.fixture
def knobs(kfmi_mod):
    """Switch the search path's process-wide test knobs (kfmi_set_split_class,
    kfmi_set_fused: their KFMI_SPLIT / KFMI_FUSED variables are read once per
    process) and put the defaults back afterwards."""
    class Knobs:
        @staticmethod
        def split(cls):
            kfmi_mod.set_split_class(int(cls) if cls else 0)

        @staticmethod
        def fused(on):
            kfmi_mod.set_fused(str(on) != "0")
    yield Knobs
    kfmi_mod.set_split_class(0)
    kfmi_mod.set_fused(True)


def pytest_collection_modifyitems(config, items):
    # OMP inside the oracle: keep CPU tests bounded on small boxes.
    os.environ.setdefault("OMP_NUM_THREADS", "8")
