"""Split files: a throughput launch (more than 256 files) cuts
every file longer than 128 KiB into a ragged head and 128 KiB segments that
separate waves checksum, every unit in address order; the segment CRCs are
folded on the GPU (crc(A||B) = shift(crc(A), |B|) ^ crc(B), the seed on the
head).  Results must be bit-identical to Func::crc (src/common/func.cpp:426-435)
whatever the split: against the oracle, and against the same context with
splitting off."""
import numpy as np
import pytest

from conftest import ocrc
from test_latency_form import _oracle_batch
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

KSEG = 128 * 1024


@pytest.fixture
def sctx(gpu_ctx):
    """The product context (the address-ordered unit list)."""
    yield gpu_ctx


def _edge_lengths():
    L = [KSEG - 1, KSEG, KSEG + 1, 2 * KSEG - 1, 2 * KSEG, 2 * KSEG + 1, 3 * KSEG + 17, 8 * KSEG, 8 * KSEG + 5,
         (1 << 20) + 12345, 3 * (1 << 20) + 7, 9 * (1 << 20) + 1]
    return L


def test_split_batch_matches_oracle_and_unsplit(sctx, oracle):
    """300+ files mixing the split edges (K*128 KiB +- 1, ragged heads of every
    size), small files and 1-9 MiB files, every alignment, seeds (compute) --
    one host batch (throughput form): oracle-exact, and equal to split off."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(3030)
    lens = _edge_lengths() * 3 + [int(x) for x in rng.integers(0, 40000, 200)] + \
        [int(x) for x in rng.integers(KSEG, 5 << 20, 80)]
    rng.shuffle(lens)
    n = len(lens)
    lens = np.array(lens, np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 16, n).astype(np.uint64))
    buf = synth_bytes(3031, int(offs[-1] + lens[-1]) + 256)
    seeds = np.where(rng.integers(0, 2, n) == 0, 0, rng.integers(0, 2**32, n)).astype(np.uint32)
    exp = _oracle_batch(oracle, buf, offs, lens, seeds)
    got = sctx.batch(buf, offs, lens, seeds)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16) for i in bad[:10]]
    c2 = crc.Context(0)
    try:
        c2.set_split(False)
        assert (c2.batch(buf, offs, lens, seeds) == exp).all()
    finally:
        c2.close()


def test_split_verify_device_wrong_expectations(sctx, oracle):
    """Device-resident verify with split files: wrong expectations on split and
    whole files alike are found exactly (n_bad, verdicts, CRCs)."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(3032)
    n = 2000
    lens = np.where(rng.integers(0, 3, n) == 0, rng.integers(KSEG, 3 << 20, n), rng.integers(0, 200000, n)).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 64, n).astype(np.uint64))
    total = int(offs[-1] + lens[-1]) + 256
    img = crc.DeviceBuffer(sctx, (total + 7) // 8 * 8)
    sctx.synth_fill_device(img, (total + 7) // 8 * 8, 3033, 0)
    host = img.download(np.uint8, total)
    exp = _oracle_batch(oracle, host, offs, lens, np.zeros(n, np.uint32))
    wrong = np.sort(rng.choice(n, 97, replace=False))
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, exp
    d["aux"][wrong] ^= 0x80000000
    dd = crc.DeviceBuffer(sctx, d.nbytes).upload(d)
    dc, dok, dnb = crc.DeviceBuffer(sctx, 4 * n), crc.DeviceBuffer(sctx, n), crc.DeviceBuffer(sctx, 4)
    try:
        assert int((lens[wrong] > KSEG).sum()) > 10
        for rep in range(2):
            dok.zero()
            dnb.zero()
            sctx.verify_device(dd, n, img, dc, dok, dnb)
            sctx.sync()
            assert int(dnb.download(np.uint32)[0]) == wrong.size, rep
            ok = dok.download(np.uint8, n)
            assert (np.nonzero(ok == 0)[0] == wrong).all() and (ok[np.setdiff1d(np.arange(n), wrong)] == 1).all()
            assert (dc.download(np.uint32, n) == exp).all(), rep
    finally:
        for b in (img, dd, dc, dok, dnb):
            b.free()


def test_split_capacity_overflow_splits_the_prefix_that_fits(sctx, oracle):
    """The plan has room for max(2n, 65,536) segments.  400 files of 9 MiB (28,400
    segments) all split; 1,000 of them need 71,000, so the longest prefix of files
    whose segments fit is split (round 4's form split nothing then) and
    the files after it stay whole -- split_stats reports exactly that prefix's
    segments.  Then 300 files of 64 MiB (153,300 segments; the first 128 fit): a
    batch of big files still spreads over the grid.  Every CRC exact."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(3034)
    for n, L in ((400, 9 * (1 << 20) + 3), (1000, 9 * (1 << 20) + 3), (300, 64 * (1 << 20) + 5)):
        src = crc.DeviceBuffer(sctx, L + 4096)
        sctx.synth_fill_device(src, (L + 4096) // 8 * 8, 3035, 0)
        host = src.download(np.uint8, L + 4096)
        offs = rng.integers(0, 4000, n).astype(np.uint64)  # overlapping files over one region
        lens = np.full(n, L - 4000, np.uint32) - rng.integers(0, 100, n).astype(np.uint32)
        seeds = rng.integers(0, 2**32, n).astype(np.uint32)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"], d["len"], d["aux"] = offs, lens, seeds
        dd = crc.DeviceBuffer(sctx, d.nbytes).upload(d)
        out = crc.DeviceBuffer(sctx, 4 * n)
        try:
            sctx.batch_device(dd, n, src, out)
            sctx.sync()
            got = out.download(np.uint32, n)
            idx = np.linspace(0, n - 1, 40).astype(np.int64)
            exp = _oracle_batch(oracle, host, offs[idx], lens[idx], seeds[idx])
            assert (got[idx] == exp).all(), n
            st = sctx.split_stats()
            K = np.where(lens > KSEG, (lens.astype(np.int64) - 1) // KSEG, 0)
            cum = np.cumsum(K)
            fit = int((cum <= st["cap"]).sum())
            assert st["files"] == n and st["cap"] == max(2 * n, 65536)
            assert st["used"] == (int(cum[fit - 1]) if fit else 0) > 0, (n, st, fit)
            assert (fit == n) == (n == 400), (n, fit)
        finally:
            dd.free()
            out.free()
            src.free()


def test_split_packet_bodies(sctx, oracle):
    """Packet frames with bodies over 128 KiB (a write of 1 MiB is one frame):
    the decode CRC (seed TFS_PACKET_FLAG_V1, base_packet.cpp:141) through the
    split launch equals the oracle's statuses and CRCs."""
    import test_packet as tp
    from tfs_amd import packet as pk
    rng = np.random.default_rng(3036)
    parts, frames, pos = [], [], 0
    for i in range(300):
        size = int(rng.integers(KSEG - 10, 3 * KSEG)) if i % 3 == 0 else int(rng.integers(1, 5000))
        body = pk.write_data_body(i, i, 0, synth_bytes(3037 + i, size).tobytes())
        f = pk.frame_v1(body, pid=i, crc=ocrc(oracle, pk.TFS_PACKET_FLAG_V1, body) ^ (1 if i % 50 == 7 else 0))
        gap = int(rng.integers(0, 4))
        parts.append(b"\0" * gap + f)
        frames.append((pos + gap, len(f)))
        pos += gap + len(f)
    raw = b"".join(parts)
    buf = np.frombuffer(raw, np.uint8)
    c, st, nbad, rc = sctx.packet_verify(buf, [f[0] for f in frames], [f[1] for f in frames])
    oc, ost, obad = tp.o_verify(oracle, buf, frames)
    assert np.array_equal(st, ost) and np.array_equal(c, oc) and nbad == obad == 6
