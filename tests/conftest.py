import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def ref_lib():
    """The reference libwebp built from /root/reference by oracle/Makefile
    (present in the dev container; travels to the GPU box as a built file)."""
    import ctypes
    from libwebp_amd import abi
    path = os.path.join(ROOT, "oracle", "_ref", "libwebp_ref.so")
    if not os.path.exists(path):
        pytest.skip("reference build oracle/_ref not present")
    return abi.bind_encoder_api(ctypes.CDLL(path))


@pytest.fixture(scope="session")
def gpu():
    import libwebp_amd
    if libwebp_amd.device_count() <= 0:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")
    return libwebp_amd
