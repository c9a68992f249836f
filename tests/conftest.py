import asyncio
import os
import sys

import pytest

# lease / wait timings of the HA tests are multiplied by this under a slow tracer (the
# coverage gate sets NEXUS_TEST_TIME_SCALE: line tracing slows the code 3-10x)
TIME_SCALE = float(os.environ.get("NEXUS_TEST_TIME_SCALE", "1") or 1)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (amd-smi / HIP); run with -m gpu")
    config.addinivalue_line("markers", "slow: multi-second integration or bench-style test")


def run(coro, timeout=60):
    """Run a coroutine on a fresh loop (tests stay plain functions, no plugin needed)."""
    return asyncio.run(asyncio.wait_for(coro, timeout))


@pytest.fixture
def arun():
    return run
