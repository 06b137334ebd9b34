import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "nk8_golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def has_gpu_device() -> bool:
    """A HIP device node exists (checked without initialising a runtime)."""
    return os.path.exists("/dev/kfd")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)
