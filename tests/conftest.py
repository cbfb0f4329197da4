import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle", "py"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    d = os.path.join(REPO, "tests", "golden")
    return {name: np.load(os.path.join(d, f"{name}_golden.npz"), allow_pickle=False)
            for name in ("msm", "ntt", "poly")}
