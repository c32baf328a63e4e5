import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tfs_amd.synth import synth_bytes  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def _build_oracle():
    so = os.path.join(ROOT, "oracle", "liboracle_crc.so")
    src = os.path.join(ROOT, "oracle", "crc_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle_crc.so"])
    return so


@pytest.fixture(scope="session")
def oracle():
    """CPU restatement (test infrastructure only)."""
    L = ctypes.CDLL(_build_oracle())
    L.oracle_crc.restype = ctypes.c_uint32
    L.oracle_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    L.oracle_datafile_get_crc.restype = ctypes.c_uint32
    L.oracle_datafile_get_crc.argtypes = [ctypes.c_char_p, ctypes.c_int32]
    L.oracle_crc_batch_mt.restype = ctypes.c_int
    L.oracle_crc_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.oracle_crc_batch.restype = None
    L.oracle_crc_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_verify_file.restype = ctypes.c_int32
    L.oracle_verify_file.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                     ctypes.POINTER(ctypes.c_uint32)]
    L.oracle_compact.restype = ctypes.c_int64
    L.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    L.oracle_loopback_block.restype = ctypes.c_int32
    L.oracle_loopback_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_packet_verify.restype = ctypes.c_uint32
    L.oracle_packet_verify.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2
    L.oracle_packet_seal.restype = None
    L.oracle_packet_seal.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2
    L.oracle_table.restype = None
    L.oracle_table.argtypes = [ctypes.c_void_p]
    return L


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "crc_vectors.json")) as f:
        return json.load(f)


def vector_input(v):
    """Reconstruct the input bytes of one golden vector."""
    if "hex" in v:
        return bytes.fromhex(v["hex"])
    if "fill" in v:
        return bytes([v["fill"]]) * v["len"]
    g = v["gen"]
    return synth_bytes(g["seed"], g["len"], g.get("offset", 0)).tobytes()


@pytest.fixture(scope="session")
def gpu_ctx():
    import tfs_amd.crc as crc
    ctx = crc.Context(0)
    yield ctx
    ctx.close()


def ocrc(oracle, seed, data, n=None):
    n = len(data) if n is None else n
    return oracle.oracle_crc(seed & 0xFFFFFFFF, bytes(data), n)
