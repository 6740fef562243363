import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pm-rl_amd"), os.path.join(ROOT, "oracle"), ROOT, os.path.dirname(__file__)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpmenv.so on cuda:0)")


@pytest.fixture(scope="session", autouse=True)
def _built_libs():
    """Build libpmenv.so / liboracle.so in place if they are missing or stale."""
    sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
    import build  # pm-rl_amd/build.py
    build.build_oracle()
    if os.path.exists("/opt/rocm/bin/hipcc"):
        build.build_pmenv()
