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


@pytest.fixture(scope="session", autouse=True)
def _heartbeat():
    """A line every 30 s into gpurun_out/pytest_heartbeat.txt while the session runs: the
    GPU pool takes a command that writes nothing for 3 minutes (stdout, stderr or files
    under gpurun_out/) for hung, and pytest holds a test's output until it ends -- the
    oracle's CPU proofs at k = 22 / 24 run for minutes."""
    import threading
    import time

    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", REPO), "gpurun_out")
    stop = threading.Event()

    def beat():
        try:
            os.makedirs(out, exist_ok=True)
        except OSError:
            return
        t0 = time.time()
        while not stop.wait(30):
            try:
                with open(os.path.join(out, "pytest_heartbeat.txt"), "a") as f:
                    f.write(f"{time.strftime('%H:%M:%S')} pytest alive, {time.time() - t0:.0f} s\n")
            except OSError:
                return

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
