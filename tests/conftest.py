import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def naive_decode():
    """The test-only lane-per-chunk Snappy decoder (tests/native/libnx_test_naive.so, built by
    __graft_entry__.build()), with nx_snappy_decode_batch's contract: a cross-check of the product
    decoder, never shipped in libnetty_amd.so."""
    import ctypes as C
    from netty_amd import _lib
    _lib.load()  # libnetty_amd.so first (the test library links against it)
    L = C.CDLL(os.path.join(ROOT, "tests", "native", "libnx_test_naive.so"))
    f = L.nx_snappy_decode_batch_naive
    f.restype = C.c_int32
    f.argtypes = [C.c_void_p] * 11 + [C.c_uint32, C.c_void_p]
    return f
