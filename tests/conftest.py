import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgraindispatch on cuda:0)")
    if os.environ.get("GD_TEST_BALLOT_RANKS") == "1":
        # the whole suite with every stable rank by ballots (GD_CFG_NO_LANE_ORDER on every handle): the
        # library's path on a device without the LDS lane order
        from orleans_amd import graindispatch
        graindispatch.FORCE_NO_LANE_ORDER = True
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
