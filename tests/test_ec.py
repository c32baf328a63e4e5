"""Erasure code: ErasureCode over jerasure's Cauchy bitmatrix.

Golden vectors (tests/golden/ec_vectors.json) come from the reference's own
jerasure.cpp/galois.cpp compiled in the build container (oracle/gen_golden_ec.py);
the CPU restatement (oracle/ec_oracle.c) is pinned to them here, and the GPU
path is compared with both.  Mirrors tests/dataserver/test_erasure_code.cpp
(coding: k=5 m=3 1 MiB, random erasures, decode restores; exception: statuses).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT
from tfs_amd.synth import synth_bytes


@pytest.fixture(scope="module")
def ec_golden():
    with open(os.path.join(ROOT, "tests", "golden", "ec_vectors.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="module")
def ec_oracle():
    so = os.path.join(ROOT, "oracle", "liboracle_ec.so")
    src = os.path.join(ROOT, "oracle", "ec_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle_ec.so"])
    L = ctypes.CDLL(so)
    L.oracle_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.oracle_ec_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_int]
    return L


def members(k, m, size, seed):
    return [synth_bytes(seed + i, size).copy() if i < k else np.zeros(size, np.uint8) for i in range(k + m)]


def ptrs(ms):
    return (ctypes.c_void_p * len(ms))(*[None if a is None else a.ctypes.data for a in ms])


def sha(a):
    return hashlib.sha256(a.tobytes()).hexdigest()


def o_encode(L, k, m, ms, size, sizes=None):
    sz = None if sizes is None else (ctypes.c_int * len(ms))(*sizes)
    return L.oracle_ec_encode(k, m, ptrs(ms), sz, size)


def o_decode(L, k, m, erased, ms, size, sizes=None):
    sz = None if sizes is None else (ctypes.c_int * len(ms))(*sizes)
    return L.oracle_ec_decode(k, m, (ctypes.c_int * (k + m))(*erased), ptrs(ms), sz, size)


def test_oracle_matches_reference_golden(ec_oracle, ec_golden):
    for c in ec_golden:
        k, m, size = c["k"], c["m"], c["size"]
        ms = members(k, m, size, c["seed"])
        assert o_encode(ec_oracle, k, m, ms, size) == 0
        for i in range(m):
            assert sha(ms[k + i]) == c["parity_sha256"][i], (k, m, i)
            assert ms[k + i][:64].tobytes().hex() == c["parity_head_hex"][i]
        coded = [a.copy() for a in ms]
        for d in c["decode"]:
            er = d["erased"]
            ms2 = [coded[i].copy() if er[i] == 0 else np.zeros(size, np.uint8) for i in range(k + m)]
            assert o_decode(ec_oracle, k, m, er, ms2, size) == d["rc"]
            for i, h in d["rebuilt_sha256"].items():
                assert sha(ms2[int(i)]) == h


def test_oracle_statuses_like_reference_test(ec_oracle):
    """test_erasure_code.cpp:150-200 (excepiton)."""
    k, m, size = 5, 3, 8192
    ms = members(k, m, size, 1)
    bad = list(ms)
    bad[0] = None
    assert o_encode(ec_oracle, k, m, bad, size) == -16001            # EXIT_DATA_INVALID
    assert o_encode(ec_oracle, k, m, ms, size + 1024, [size] * 8) == -16001
    assert o_encode(ec_oracle, k, m, ms, size - 100) == -16002       # EXIT_SIZE_INVALID
    assert o_decode(ec_oracle, k, m, [0, 0, 0, 1, 1, 1, 0, 1], ms, size) == -16004  # EXIT_NO_ENOUGH_DATA
    assert o_decode(ec_oracle, k, m, [0, 0, 0, 0, 1, 0, 1, 1], ms, size) == 0


# ---------------------------------------------------------------- GPU --------

@pytest.mark.gpu
def test_gpu_encode_decode_golden(gpu_ctx, ec_golden):
    from tfs_amd.ec import ErasureCode
    for c in ec_golden:
        k, m, size = c["k"], c["m"], c["size"]
        ms = members(k, m, size, c["seed"])
        enc = ErasureCode(gpu_ctx, k, m)
        assert enc.rc == 0 and enc.encode(ms, size) == 0
        for i in range(m):
            assert sha(ms[k + i]) == c["parity_sha256"][i], (k, m, i)
        enc.free()
        for d in c["decode"]:
            er = d["erased"]
            ms2 = [ms[i].copy() if er[i] == 0 else np.zeros(size, np.uint8) for i in range(k + m)]
            dec = ErasureCode(gpu_ctx, k, m, er)
            assert dec.rc == d["rc"]
            if d["rc"] == 0:
                assert dec.decode(ms2, size) == 0
                for i, h in d["rebuilt_sha256"].items():
                    assert sha(ms2[int(i)]) == h, (k, m, er, i)
            dec.free()


@pytest.mark.gpu
def test_gpu_coding_like_reference_test(gpu_ctx, ec_oracle):
    """test_erasure_code.cpp:61-133 (coding): k=5 m=3, 1 MiB members, 3 erased."""
    from tfs_amd.ec import ErasureCode
    k, m, size = 5, 3, 1 << 20
    rng = np.random.default_rng(7)
    ms = [rng.integers(0, 128, size, dtype=np.uint8) for _ in range(k + m)]  # rand() % 128 as the test
    enc = ErasureCode(gpu_ctx, k, m)
    assert enc.encode(ms, size) == 0
    oms = [a.copy() for a in ms]
    for i in range(k, k + m):
        oms[i][:] = 0
    assert o_encode(ec_oracle, k, m, oms, size) == 0
    for i in range(k, k + m):
        assert (ms[i] == oms[i]).all()
    for trial in range(6):
        dead = sorted(rng.choice(k + m, 3, replace=False).tolist())
        er = [1 if i in dead else 0 for i in range(k + m)]
        src = [ms[i].copy() for i in range(k + m)]
        work = [np.zeros(size, np.uint8) if er[i] else ms[i].copy() for i in range(k + m)]
        dec = ErasureCode(gpu_ctx, k, m, er)
        assert dec.rc == 0 and dec.decode(work, size) == 0
        for i in dead:
            assert (work[i] == src[i]).all(), (dead, i)
        dec.free()


@pytest.mark.gpu
def test_gpu_statuses_and_device_form(gpu_ctx, ec_oracle):
    import tfs_amd.crc as crc
    from tfs_amd.ec import ErasureCode
    k, m, size = 5, 3, 8192
    enc = ErasureCode(gpu_ctx, k, m)
    ms = members(k, m, size, 9)
    bad = list(ms)
    bad[0] = None
    assert enc.encode(bad, size) == -16001
    assert enc.encode(ms, size + 1024, sizes=[size] * 8) == -16001
    assert enc.encode(ms, size - 100) == -16002
    assert enc.decode(ms, size) == -16003            # no decoding matrix configured
    assert ErasureCode(gpu_ctx, k, m, [0, 0, 0, 1, 1, 1, 0, 1]).rc == -16004
    # device-resident form, 4 MiB members, every erasure pattern of 2 data + 1 parity
    size = 4 << 20
    host = members(k, m, size, 21)
    d = [crc.DeviceBuffer(gpu_ctx, size).upload(h) for h in host]
    assert enc.encode_device(d, size) == 0
    gpu_ctx.sync()
    o = [h.copy() for h in host]
    assert o_encode(ec_oracle, k, m, o, size) == 0
    for i in range(k, k + m):
        assert (d[i].download(np.uint8, size) == o[i]).all()
    er = [1, 0, 1, 0, 0, 0, 1, 0]
    for i in (0, 2, 6):
        d[i].zero()
    dec = ErasureCode(gpu_ctx, k, m, er)
    assert dec.decode_device(d, size) == 0
    gpu_ctx.sync()
    for i in (0, 2, 6):
        assert (d[i].download(np.uint8, size) == o[i]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6])
def test_gpu_kernel_forms_ragged_sizes(gpu_ctx, ec_oracle, variant, monkeypatch):
    """Every kernel form (TFS_EC_VARIANT 0: one grid step of tiles per wave; 1-3:
    chunks of 2, 4, 8 tiles per wave step with the cross-tile prefetch; 4, 6: the
    tile kernel striding over 8,192 / 2,048 workgroups) on unit counts that leave
    partial tiles, partial chunks and a grid stride larger than the work:
    encode and a 3-member decode byte-exact against the oracle.  The forms live
    in the measurement build (the product library never
    reads TFS_EC_VARIANT), so a variant runs on a measurement-build context."""
    import tfs_amd.crc as crc
    from tfs_amd.ec import ErasureCode
    monkeypatch.setenv("TFS_EC_VARIANT", str(variant))
    vctx = crc.Context(0, measure=True) if variant else gpu_ctx
    try:
        _ec_forms_case(vctx, ec_oracle, variant)
    finally:
        if variant:
            vctx.close()


def _ec_forms_case(gpu_ctx, ec_oracle, variant):
    from tfs_amd.ec import ErasureCode
    k, m = 5, 3
    for units in (1, 3, 5, 17, 33, 1031, 70001):
        size = units * 1024
        ms = members(k, m, size, 500 + units)
        enc = ErasureCode(gpu_ctx, k, m)
        assert enc.encode(ms, size) == 0
        o = [a.copy() for a in ms]
        for i in range(k, k + m):
            o[i][:] = 0
        assert o_encode(ec_oracle, k, m, o, size) == 0
        for i in range(k, k + m):
            assert (ms[i] == o[i]).all(), (variant, units, i)
        er = [0, 1, 0, 0, 1, 0, 0, 1]
        work = [np.zeros(size, np.uint8) if er[i] else ms[i].copy() for i in range(k + m)]
        dec = ErasureCode(gpu_ctx, k, m, er)
        assert dec.rc == 0 and dec.decode(work, size) == 0
        for i in (1, 4, 7):
            assert (work[i] == ms[i]).all(), (variant, units, i)
        enc.free()
        dec.free()
