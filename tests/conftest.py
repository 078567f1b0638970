import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")
# gloo ranks of the multi-process tests talk over loopback: no host-name lookup (the container's
# name may not resolve; a slow lookup under load once stalled a two-rank test past its timeout)
os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
