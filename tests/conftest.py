import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle_crc32.so")
GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment (run with -m gpu on an MI355X)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def _build_if_missing():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    so = os.path.join(ROOT, "ambry_amd", "libambrycrc.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ambry_amd")], check=True, capture_output=True)


class Oracle:
    """ctypes view of oracle/build/liboracle_crc32.so (test infrastructure)."""

    def __init__(self, path=ORACLE_SO):
        L = ctypes.CDLL(path)
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_crc32.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_crc32_bytewise.restype = ctypes.c_uint32
        L.oracle_crc32_bytewise.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_crc32_combine.restype = ctypes.c_uint32
        L.oracle_crc32_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_crc32_tables.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_crc32_reset.argtypes = [ctypes.c_void_p]
        L.oracle_crc32_get_value.restype = ctypes.c_uint64
        L.oracle_crc32_get_value.argtypes = [ctypes.c_void_p]
        L.oracle_crc32_update_bytes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        L.oracle_crc32_update_byte.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_crc32_batch.restype = ctypes.c_int
        L.oracle_crc32_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_zlib_batch.restype = ctypes.c_int
        L.oracle_zlib_batch.argtypes = L.oracle_crc32_batch.argtypes
        self.L = L

    @staticmethod
    def _p(data):
        import numpy as np

        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                 else data)
        return a, a.ctypes.data_as(ctypes.c_void_p)

    def crc32(self, data, crc=0):
        a, p = self._p(data)
        return self.L.oracle_crc32(crc, p, a.nbytes)

    def crc32_bytewise(self, data, crc=0):
        a, p = self._p(data)
        return self.L.oracle_crc32_bytewise(crc, p, a.nbytes)

    def combine(self, c1, c2, len2):
        return self.L.oracle_crc32_combine(c1, c2, len2)

    def batch(self, mem, off, length, crc_in=None, threads=1, zlib=False):
        """Per-chunk CRCs on the CPU: the Crc32.java restatement, or (zlib=True) the system zlib."""
        import numpy as np

        mem = np.ascontiguousarray(mem)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        out = np.zeros(len(off), dtype=np.uint32)
        cin = None if crc_in is None else np.ascontiguousarray(crc_in, dtype=np.uint32)
        fn = self.L.oracle_zlib_batch if zlib else self.L.oracle_crc32_batch
        rc = fn(mem.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p),
                                       length.ctypes.data_as(ctypes.c_void_p),
                                       None if cin is None else cin.ctypes.data_as(ctypes.c_void_p),
                                       out.ctypes.data_as(ctypes.c_void_p), len(off), threads)
        assert rc == 0
        return out


@pytest.fixture(scope="session")
def oracle():
    _build_if_missing()
    return Oracle()


@pytest.fixture(scope="session")
def ambry():
    _build_if_missing()
    import ambry_amd

    ambry_amd.lib()
    return ambry_amd


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "crc32_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def fingerprint():
    with open(os.path.join(GOLDEN, "crc32_table_fingerprint.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    """Initialises libambrycrc on cuda:0; the tests using it are marked gpu."""
    import torch

    _build_if_missing()
    from ambry_amd import device

    torch.cuda.init()
    device.init(0)
    # the GPU suite tests the GPU leg of the *_host entries; the host-resident dispatch policy's own
    # tests (test_host_policy.py, test_gpu_host_policy) set it themselves
    device.set_host_policy(0, device.HOST_GPU)
    return device
