"""Packet CRC: BasePacket's body CRC with seed TFS_PACKET_FLAG_V1.

Reference behaviour restated by oracle/crc_oracle.c (oracle_packet_*):
getPacketInfo (base_packet_streamer.cpp:43-124), decode (base_packet.cpp:100-170),
copy/reply (:74,208).  The reference's own test (tests/common/test_packet.cpp:
124-197, encode_and_decode) serializes a message, sets crc = Func::crc(
TFS_PACKET_FLAG_V1, body), writes a V1 header and decodes it back; the tests here
follow that flow with WriteDataMessage bodies (the hot packet of the write path).
CPU tests pin the oracle; GPU tests compare the C ABI with it frame by frame.
"""
import struct
import zlib

import numpy as np
import pytest

from tfs_amd import packet as pk
from tfs_amd.synth import synth_bytes

SEED = pk.TFS_PACKET_FLAG_V1


def zlib_func_crc(seed, data):
    """Independent restatement: Func::crc(c, d) == ~zlib.crc32(d, ~c)."""
    return (~zlib.crc32(bytes(data), (~seed) & 0xFFFFFFFF)) & 0xFFFFFFFF


def o_verify(oracle, buf, frames):
    off = np.array([f[0] for f in frames], np.uint64)
    av = np.array([f[1] for f in frames], np.uint32)
    crc = np.zeros(len(frames), np.uint32)
    st = np.zeros(len(frames), np.int32)
    b = np.frombuffer(bytes(buf), np.uint8).copy()
    bad = oracle.oracle_packet_verify(b.ctypes.data, off.ctypes.data, av.ctypes.data, len(frames), crc.ctypes.data,
                                      st.ctypes.data)
    return crc, st, bad


def o_seal(oracle, buf, frames):
    off = np.array([f[0] for f in frames], np.uint64)
    av = np.array([f[1] for f in frames], np.uint32)
    crc = np.zeros(len(frames), np.uint32)
    st = np.zeros(len(frames), np.int32)
    b = np.frombuffer(bytes(buf), np.uint8).copy()
    oracle.oracle_packet_seal(b.ctypes.data, off.ctypes.data, av.ctypes.data, len(frames), crc.ctypes.data,
                              st.ctypes.data)
    return b, crc, st


def build_stream(rng, n=60):
    """A mixed stream of frames covering every branch of getPacketInfo/decode.
    Returns (bytes, [(offset, avail)], expected-kind list)."""
    parts, frames, kinds = [], [], []
    pos = 0

    def add(raw, avail=None, kind=""):
        nonlocal pos
        # random 0..7 bytes of gap so frames start at every alignment
        gap = int(rng.integers(0, 8))
        parts.append(b"\xAA" * gap)
        pos += gap
        parts.append(raw)
        frames.append((pos, len(raw) if avail is None else avail))
        kinds.append(kind)
        pos += len(raw)

    def sealed(body, version=pk.TFS_PACKET_VERSION_V2, pcode=pk.WRITE_DATA_MESSAGE):
        return pk.frame_v1(body, pcode=pcode, version=version, pid=7, crc=zlib_func_crc(SEED, body))

    for i in range(n):
        ln = int(rng.choice([1, 3, 15, 16, 17, 31, 32, 33, 100, 1000, 4095, 4096, 65536, 65537]))
        data = synth_bytes(1000 + i, ln).tobytes()
        body = pk.write_data_body(0x1234 + i, 0xABCDEF00 + i, 0, data, ds=[11, 12, 13], lease=(3, 77 + i))
        add(sealed(body), kind="ok")
    body = pk.write_data_body(9, 9, 0, synth_bytes(5, 70000).tobytes())
    good = bytearray(sealed(body))
    add(bytes(good), kind="ok")
    bad_body = bytearray(good)
    bad_body[24 + 5000] ^= 0x10
    add(bytes(bad_body), kind="crc")
    bad_crc = bytearray(good)
    bad_crc[21] ^= 0x01
    add(bytes(bad_crc), kind="crc")
    add(sealed(b"123456789"), kind="ok")                                      # KAT body
    add(pk.frame_v1(b"x" * 40, version=0, crc=0xDEAD), kind="nocheck")        # V1 flag, version 0
    add(pk.header_v1(40, -5, 0, 1, zlib_func_crc(SEED, b"y" * 40)) + b"y" * 40, kind="ok")  # negative type
    add(pk.header_v0(40, 9) + b"z" * 40, kind="nocheck")                      # V0 frame
    v0neg_body = struct.pack("<QI", 5, zlib_func_crc(SEED, b"w" * 28)) + b"w" * 28
    add(pk.header_v0(40, -9) + v0neg_body, kind="ok")                          # V0, negative type quirk
    add(pk.header_v0(8, -9) + b"q" * 8, kind="broken")                        # ... too short for id/crc
    add(struct.pack("<IihhQI", 0x12345678, 40, 9, 2, 1, 0) + b"u" * 40, kind="broken")  # bad flag
    add(pk.header_v1(0, 9, 2, 1) + b"", kind="broken")                          # length 0
    add(pk.header_v1(-4, 9, 2, 1) + b"", kind="broken")                         # negative length
    add(pk.header_v1(0x4000001, 9, 2, 1), kind="broken")                        # > 64 MiB
    add(pk.header_v1(0x4000000, 9, 2, 1), kind="incomplete")                    # max length, body absent
    add(sealed(b"v" * 100)[:60], kind="incomplete")                              # body cut
    add(sealed(b"v" * 100)[:20], kind="incomplete")                              # V1 header cut
    add(b"TFSN"[::-1] + b"\x01\x00", kind="incomplete")                         # < 12 bytes
    return b"".join(parts), frames, kinds


KIND_STATUS = {"ok": 0, "nocheck": 0, "crc": -1010, "broken": -1, "incomplete": 1}


def test_oracle_packet_kat(oracle):
    # crc(0x4E534654, "123456789") = 0xCADE6EAE  (SURVEY §8c known answer)
    fr = pk.frame_v1(b"123456789")
    b, crc, st = o_seal(oracle, fr, [(0, len(fr))])
    assert st[0] == 0 and crc[0] == 0xCADE6EAE
    assert struct.unpack_from("<I", b.tobytes(), 20)[0] == 0xCADE6EAE
    c2, st2, bad = o_verify(oracle, b.tobytes(), [(0, len(fr))])
    assert bad == 0 and st2[0] == 0 and c2[0] == 0xCADE6EAE


def test_oracle_packet_branches(oracle):
    rng = np.random.default_rng(3)
    buf, frames, kinds = build_stream(rng, n=12)
    crc, st, bad = o_verify(oracle, buf, frames)
    for i, k in enumerate(kinds):
        assert st[i] == KIND_STATUS[k], (i, k, st[i])
    assert bad == sum(1 for k in kinds if KIND_STATUS[k] != 0)
    # the computed CRCs of checked frames equal the zlib identity
    for i, (o, a) in enumerate(frames):
        if kinds[i] in ("ok", "crc") and buf[o:o + 4] == struct.pack("<I", SEED):
            body = buf[o + 24:o + a]
            assert crc[i] == zlib_func_crc(SEED, body)


def test_split_frames_walks_stream():
    bodies = [pk.write_data_body(1, i, 0, bytes([i]) * (i * 37 + 1)) for i in range(20)]
    stream = b"".join(pk.frame_v1(b) for b in bodies) + pk.header_v0(5, 3) + b"abcde"
    fr = pk.split_frames(stream)
    assert len(fr) == 21
    assert all(a == 24 + len(b) for (o, a), b in zip(fr, bodies))
    assert fr[-1][1] == 17 and fr[-1][0] + 17 == len(stream)
    # truncated tail -> incomplete last frame
    fr2 = pk.split_frames(stream[:-3])
    assert fr2[-1][1] == 14


@pytest.mark.gpu
def test_gpu_packet_verify_matches_oracle(gpu_ctx, oracle):
    rng = np.random.default_rng(11)
    buf, frames, kinds = build_stream(rng)
    crc, st, nbad, rc = gpu_ctx.packet_verify(buf, [f[0] for f in frames], [f[1] for f in frames])
    ocrc_, ost, obad = o_verify(oracle, buf, frames)
    assert np.array_equal(st, ost)
    assert np.array_equal(crc, ocrc_)
    assert nbad == obad and rc == (-1010 if obad else 0)
    for i, k in enumerate(kinds):
        assert st[i] == KIND_STATUS[k], (i, k)


@pytest.mark.gpu
def test_gpu_packet_seal_then_verify(gpu_ctx, oracle):
    rng = np.random.default_rng(12)
    parts, frames, pos = [], [], 0
    for i in range(300):
        ln = int(rng.integers(1, 200000)) if i % 10 == 0 else int(rng.integers(1, 5000))
        body = pk.write_data_body(i, i, 0, synth_bytes(i, ln).tobytes(), ds=[1, 2])
        fr = pk.frame_v1(body, pid=i)  # crc 0: unsealed
        gap = int(rng.integers(0, 5))
        parts.append(b"\0" * gap + fr)
        frames.append((pos + gap, len(fr)))
        pos += gap + len(fr)
    raw = b"".join(parts)
    ob, ocrc_, ost = o_seal(oracle, raw, frames)
    buf = np.frombuffer(raw, np.uint8).copy()
    crc, st = gpu_ctx.packet_seal(buf, [f[0] for f in frames], [f[1] for f in frames])
    assert np.array_equal(st, ost) and np.array_equal(crc, ocrc_)
    assert np.array_equal(buf, ob)  # identical sealed bytes
    crc2, st2, nbad, rc = gpu_ctx.packet_verify(buf, [f[0] for f in frames], [f[1] for f in frames])
    assert nbad == 0 and rc == 0 and np.array_equal(crc2, crc)


@pytest.mark.gpu
@pytest.mark.parametrize("n_ok,form", [(200, "small"), (600, "one_pass"), (600, "three")])
def test_gpu_packet_device_resident(gpu_ctx, oracle, n_ok, form, monkeypatch):
    """Device-resident verify then seal of a stream with every status kind, at both
    launch sizes: <= 256 frames (parse, latency form, finish) and more (round 5's
    one-pass packet_files_kernel; `three`: the measurement build's three-launch
    form of the same launch, TFS_CRC_VARIANT=51).  Statuses, CRCs, n_bad and the
    sealed bytes equal the oracle's."""
    import tfs_amd.crc as crc_mod
    if form == "three":
        monkeypatch.setenv("TFS_CRC_VARIANT", "51")
        gpu_ctx = crc_mod.Context(0)
        monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    rng = np.random.default_rng(13)
    buf, frames, kinds = build_stream(rng, n=n_ok)
    n = len(frames)
    d = np.zeros(n, crc_mod.PACKET_DESC_DTYPE)
    d["offset"] = [f[0] for f in frames]
    d["len"] = [f[1] for f in frames]
    b = np.frombuffer(buf, np.uint8)
    d_base = crc_mod.DeviceBuffer(gpu_ctx, len(b) + 16).upload(b)
    d_desc = crc_mod.DeviceBuffer(gpu_ctx, d.nbytes).upload(d)
    d_crc = crc_mod.DeviceBuffer(gpu_ctx, 4 * n)
    d_st = crc_mod.DeviceBuffer(gpu_ctx, 4 * n)
    d_bad = crc_mod.DeviceBuffer(gpu_ctx, 4)
    d_bad.zero()
    gpu_ctx.packet_verify_device(d_desc, n, d_base, d_crc, d_st, d_bad)
    gpu_ctx.sync()
    ocrc_, ost, obad = o_verify(oracle, buf, frames)
    assert np.array_equal(d_st.download(np.int32, n), ost)
    assert np.array_equal(d_crc.download(np.uint32, n), ocrc_)
    assert int(d_bad.download(np.uint32, 1)[0]) == obad
    # seal on the device: the resident frames get their header crc rewritten
    gpu_ctx.packet_seal_device(d_desc, n, d_base, d_crc, d_st)
    gpu_ctx.sync()
    ob, _, _ = o_seal(oracle, buf, frames)
    assert np.array_equal(d_base.download(np.uint8, len(b)), ob)
    if form == "three":
        gpu_ctx.close()


@pytest.mark.gpu
def test_ds_packet_codec_roundtrip(gpu_ctx, oracle):
    """The C++ codec (tfs_amd/ds/packet_codec.cpp): a send batch sealed on the GPU
    decodes cleanly; a flipped body byte fails that frame only; a cut stream
    leaves the incomplete tail unconsumed (getPacketInfo waits for it)."""
    from tfs_amd import dataserver as ds
    enc = ds.PacketEncoder(gpu_ctx)
    bodies = []
    for i in range(40):
        body = pk.write_data_body(100 + i, 5000 + i, i * 65536, synth_bytes(77 + i, 1 + 1733 * i).tobytes(),
                                  ds=[1, 2, 3], lease=(2, 900 + i))
        bodies.append(body)
        enc.add(pk.WRITE_DATA_MESSAGE, pk.TFS_PACKET_VERSION_V2, 1000 + i, body)
    assert enc.flush() == 0
    out = enc.output()
    # identical to building the frames in Python and sealing with the oracle
    ref = b"".join(pk.frame_v1(b, version=2, pid=1000 + i) for i, b in enumerate(bodies))
    frames = pk.split_frames(ref)
    ob, _, _ = o_seal(oracle, ref, frames)
    assert out == ob.tobytes()
    rc, off, st, crc, consumed = ds.decode_stream(gpu_ctx, out)
    assert rc == 0 and len(st) == 40 and (st == 0).all() and consumed == len(out)
    bad = bytearray(out)
    bad[off[7] + 24 + 50] ^= 0x40
    rc, off2, st2, _, consumed = ds.decode_stream(gpu_ctx, bytes(bad))
    assert rc == -1010 and st2[7] == -1010 and (np.delete(st2, 7) == 0).all()
    cut = out[:off[30] + 100]
    rc, off3, st3, _, consumed = ds.decode_stream(gpu_ctx, cut)
    assert rc == 0 and consumed == off[30] and st3[-1] == 1 and len(st3) == 31
    enc.free()


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["small_host_parse", "launched"])
def test_gpu_packet_small_batches_both_paths(monkeypatch, oracle, path):
    """Batches of <= 256 frames within 8 MiB take the small path (headers walked on
    the host, bodies through the synchronous small-batch CRC); TFS_CRC_VARIANT=20
    keeps the launched parse/CRC/finish path.  Both give the oracle's statuses,
    CRCs and sealed bytes on the every-branch stream and on a seal batch."""
    import tfs_amd.crc as crc_mod
    monkeypatch.setenv("TFS_CRC_VARIANT", "20" if path == "launched" else "0")
    ctx = crc_mod.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    try:
        rng = np.random.default_rng(21)
        buf, frames, kinds = build_stream(rng, n=40)
        assert len(frames) <= 256
        crc, st, nbad, rc = ctx.packet_verify(buf, [f[0] for f in frames], [f[1] for f in frames])
        ocrc_, ost, obad = o_verify(oracle, buf, frames)
        assert np.array_equal(st, ost) and np.array_equal(crc, ocrc_)
        assert nbad == obad and rc == (-1010 if obad else 0)
        parts, fr2, pos = [], [], 0
        for i in range(100):
            body = pk.write_data_body(i, i, 0, synth_bytes(300 + i, int(rng.integers(1, 40000))).tobytes())
            f = pk.frame_v1(body, pid=i, version=int(rng.integers(0, 3)))
            gap = int(rng.integers(0, 5))
            parts.append(b"\0" * gap + f)
            fr2.append((pos + gap, len(f)))
            pos += gap + len(f)
        raw = b"".join(parts)
        ob, ocrc2, ost2 = o_seal(oracle, raw, fr2)
        b2 = np.frombuffer(raw, np.uint8).copy()
        c2, s2 = ctx.packet_seal(b2, [f[0] for f in fr2], [f[1] for f in fr2])
        assert np.array_equal(s2, ost2) and np.array_equal(c2, ocrc2) and np.array_equal(b2, ob)
        # only V0 / version-0 frames: nothing to check on the GPU
        v0 = pk.header_v0(40, 9) + b"z" * 40
        c3, s3, nb3, rc3 = ctx.packet_verify(v0, [0], [len(v0)])
        assert rc3 == 0 and nb3 == 0 and s3[0] == 0 and c3[0] == 0
    finally:
        ctx.close()
