import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def engine_gpu():
    from cadence_amd import engine
    # torch (device memory for the tests) ships its own HIP/HSA runtime beside the one
    # libcdr.so links (/opt/rocm): both load into the process, and torch's finds no GPU
    # when libcdr's initialised the device first, so torch goes first whatever test runs first
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    e = engine.Engine(0)
    yield e
    e.close()
