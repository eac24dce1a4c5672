import os
import sys

import pytest

# before any test initialises the GPU: ROCm's graph packet capture off, as the entry points start it
# (ppo_continuous_action_isaacgym.py disable_graph_packet_capture)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
