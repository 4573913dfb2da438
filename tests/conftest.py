import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(REPO, "tests", "golden", "md5_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch.device("cuda:0")
