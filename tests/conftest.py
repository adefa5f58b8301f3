import os
import sys

import pytest

# torch (device memory for the GPU tests) ships its own HIP runtime whose soname is the
# one libcdr.so links (libamdhip64.so.7): loaded first, it is the one runtime of the
# process and libcdr.so binds to it; loaded after libcdr.so it is a second runtime that
# finds no GPU once libcdr.so's has opened the device.  So torch is imported before any
# test module loads libcdr.so.
try:
    import torch  # noqa: F401
except ImportError:  # the CPU suite does not need it
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def engine_gpu():
    from cadence_amd import abi, engine
    e = engine.Engine(0)
    # the parity suite runs the class-decomposed kernel wherever it applies: the
    # host-buffer calls pack class-sorted blocks (the product default leaves them to
    # device-resident batches, cdr.h CDR_CLS_ON); tests switch it off where they compare
    e.set_cls(abi.CLS_BUILD)
    yield e
    e.close()
