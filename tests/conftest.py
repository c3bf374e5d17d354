import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The tests switch kernel paths through librthx's environment knobs
# (RTHX_NO_AXIS, RTHX_FORCE_HASH, RTHX_LB_WAIT_US, ...), which the library
# honours only with RTHX_DEV_KNOBS=1 set before it first reads one
# (rthx_common.h knob).
os.environ["RTHX_DEV_KNOBS"] = "1"
for p in (os.path.join(ROOT, "raytraceheattransfer.jl_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    yield


@pytest.fixture(scope="session")
def hip():
    """The product library on a GPU box (tests marked gpu only)."""
    from rthx import _lib

    lib = _lib.load()
    # the library under test was built from the sources in this tree (a stale
    # prebuilt librthx.so fails here, loudly)
    print(f"librthx build id {_lib.check_build_id()}")
    assert _lib.device_count() >= 1, "no HIP device visible"
    return _lib
