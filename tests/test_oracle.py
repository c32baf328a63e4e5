"""The oracle (CPU restatement, test infrastructure) pinned against the golden
vectors generated from the reference's own Func::crc text (oracle/gen_golden.py)."""
import ctypes
import os
import zlib

import numpy as np
import pytest

from conftest import ROOT, ocrc, vector_input
from tfs_amd.synth import synth_bytes


def test_golden_vectors(oracle, golden):
    for v in golden["vectors"]:
        data = vector_input(v)
        n = v.get("len_arg", len(data))
        assert ocrc(oracle, v["seed"], data, n) == v["expected"], v["name"]


def test_table_matches_reference(oracle, golden):
    tab = np.zeros(256, np.uint32)
    oracle.oracle_table(tab.ctypes.data)
    ref = {v["name"]: v["expected"] for v in golden["vectors"] if v["name"].startswith("table_")}
    assert len(ref) == 256
    for b in range(256):
        assert int(tab[b]) == ref["table_%03d" % b]


def test_continuation_vectors(oracle, golden):
    for v in golden["continuation"]:
        d = vector_input(v)
        c1 = ocrc(oracle, v["seed"], d[:v["cut"]])
        assert c1 == v["expected_first"], v["name"]
        assert ocrc(oracle, c1, d[v["cut"]:]) == v["expected"], v["name"]


def test_datafile_get_crc_big(oracle, golden):
    for v in golden["datafile_big"]:
        d = vector_input(v)
        assert oracle.oracle_datafile_get_crc(d, len(d)) == v["expected"], v["name"]


def test_zlib_identity_random(oracle):
    rng = np.random.default_rng(1)
    for _ in range(200):
        n = int(rng.integers(0, 2000))
        s = int(rng.integers(0, 2**32))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert ocrc(oracle, s, d) == (~zlib.crc32(d, (~s) & 0xFFFFFFFF)) & 0xFFFFFFFF


def test_reference_build_agrees_when_present(oracle, golden):
    so = os.path.join(ROOT, "oracle", "_ref", "libref_crc.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built (no /root/reference on this host)")
    ref = ctypes.CDLL(so)
    ref.ref_func_crc.restype = ctypes.c_uint32
    ref.ref_func_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    rng = np.random.default_rng(2)
    for _ in range(100):
        n = int(rng.integers(-3, 5000))
        d = rng.integers(0, 256, max(n, 0), dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert ref.ref_func_crc(s, d, n) == ocrc(oracle, s, d, n)


def test_loopback_block_and_verify(oracle):
    n, ln = 16, 4096
    pay = synth_bytes(0x9E3779B97F4A7C15 & 0xFFFFFFFF, n * ln)
    client = np.array([ocrc(oracle, 0, pay[i * ln:(i + 1) * ln].tobytes()) for i in range(n)], np.uint32)
    stage = np.zeros(ln, np.uint8)
    image = np.zeros(n * (ln + 36), np.uint8)
    stored = np.zeros(n, np.uint32)
    bad = oracle.oracle_loopback_block(pay.ctypes.data, n, ln, client.ctypes.data, stage.ctypes.data,
                                       image.ctypes.data, stored.ctypes.data)
    assert bad == 0 and (stored == client).all()
    client[3] ^= 1
    assert oracle.oracle_loopback_block(pay.ctypes.data, n, ln, client.ctypes.data, stage.ctypes.data,
                                        image.ctypes.data, stored.ctypes.data) == 1
