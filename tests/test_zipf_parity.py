"""The Zipf line's production launch under parity.

BASELINE configs[2] packs Zipf(1.1)-sized files (len = 4096 k + U[0, 4095], k in
1..255) FileInfo|payload into 64 MiB blocks, so payloads start at arbitrary byte
offsets and 27 % of the files are longer than 128 KiB.  At production size the
file kernel's launch then runs everything at once:

- the split plan (split_ao_count / _scan / _write): every file > 128 KiB cut into
  a ragged head and whole 128 KiB segments, every unit listed in address order;
- chunked dynamic tickets (FileCursor, CF = 4, the last units >> 3 one by one):
  taken only when the units (files + segments) come to >= 16 tickets per wave;
- the fold (split_ao_fold_kernel) joining each split file's head and segment CRCs.

Here 320 blocks of bench.zipf_sizes (~154 k files, ~118 k segments, ~93 k
tickets on 4,096 waves: the chunked path) are device-resident and run in both
forms, each checked file by file against the oracle over the device's own bytes:

- compute with mixed seeds (a third zero, the rest random);
- verify with 1,000 wrong expectations, >= 300 of them on split files:
  n_bad == 1,000, verdict 0 at exactly those files, CRCs equal to the oracle's.

tfs_crc32_split_stats proves the launch took that path (the plan split files;
units / tickets from the plan's own count).  A third test runs split launches on
two streams of one context at once (one plan per owned scheduler slot) and
checks them.

References: Func::crc src/common/func.cpp:426-435; the running-seed identity the
fold relies on, DataFile::get_crc src/dataserver/data_file.cpp:183-186; the
verify call site sync_backup.cpp:345-435.
"""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu

THREADS = 16
SEG = 128 * 1024
NBLOCKS = 320


@pytest.fixture
def sctx(gpu_ctx):
    """The product context (the address-ordered unit list)."""
    yield gpu_ctx


def _oracle_mt(oracle, host, offs, lens, seeds):
    import tfs_amd.crc as crc
    d = np.zeros(len(offs), crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, seeds
    out = np.zeros(len(offs), np.uint32)
    assert oracle.oracle_crc_batch_mt(d.ctypes.data, len(offs), host.ctypes.data, out.ctypes.data, THREADS) == 0
    return out


def _tickets(units):
    """FileCursor::init (tfs_crc_kernels.hip): chunks of 4 units, the last units >> 3 one by one."""
    nA = (units - (units >> 3)) // 4
    return nA + (units - nA * 4)


@pytest.fixture(scope="module")
def zipf_image(gpu_ctx, oracle):
    """The bench's configs[2] layout (bench_zipf): block b at b * 64 MiB, records packed from its start."""
    import tfs_amd.crc as crc
    blocks = bench.zipf_sizes(4242, NBLOCKS)
    offs, lens = [], []
    for b, L in enumerate(blocks):
        rec = np.concatenate([[0], np.cumsum(36 + L)[:-1]])
        offs.append(b * (64 << 20) + rec + 36)
        lens.append(L)
    offs = np.concatenate(offs).astype(np.uint64)
    lens = np.concatenate(lens).astype(np.uint32)
    total = max(NBLOCKS * (64 << 20), (int(offs[-1]) + int(lens[-1]) + 8191) // 4096 * 4096)
    img = crc.DeviceBuffer(gpu_ctx, total)
    gpu_ctx.synth_fill_device(img, total, 0x21FF, 0)
    gpu_ctx.sync()
    host = img.download(np.uint8, total)
    crc0 = _oracle_mt(oracle, host, offs, lens, np.zeros(len(lens), np.uint32))
    yield img, host, offs, lens, crc0
    img.free()


def test_zipf_production_launch_compute_with_seeds(sctx, oracle, zipf_image):
    import tfs_amd.crc as crc
    img, host, offs, lens, crc0 = zipf_image
    n = len(lens)
    big = lens > SEG
    assert 0.2 < big.mean() < 0.35 and lens.max() > 900 * 1024
    rng = np.random.default_rng(77)
    seeds = np.where(rng.integers(0, 3, n) == 0, 0, rng.integers(1, 2**32, n)).astype(np.uint32)
    seeds[np.nonzero(big)[0][:200]] = 0xFFFFFFFF  # all-ones seed on some split files
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, seeds
    d_d = crc.DeviceBuffer(sctx, d.nbytes).upload(d)
    d_out = crc.DeviceBuffer(sctx, 4 * n)
    try:
        sctx.batch_device(d_d, n, img, d_out)
        st = sctx.split_stats()
        got = d_out.download(np.uint32, n)
        exp = _oracle_mt(oracle, host, offs, lens, seeds)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16, int(seeds[i])) for i in bad[:10]]
        # the launch really took the production path: a plan that split every file > 128 KiB, and
        # chunked dynamic tickets over its files + ext units
        K = np.where(big, (lens.astype(np.int64) - 1) // SEG, 0)
        waves = st["grid"] * 16
        assert st["files"] == n and st["used"] == int(K.sum()) and st["used"] <= st["cap"], st
        assert st["units"] == n + int(K.sum()), st
        assert 8 <= st["grid"] <= 256 and st["launches"] >= 1
        assert _tickets(st["units"]) >= 16 * waves, (st, _tickets(st["units"]))  # kDynMinPerWave over chunks
    finally:
        d_d.free()
        d_out.free()


def test_zipf_production_launch_verify_wrong_expectations(sctx, oracle, zipf_image):
    import tfs_amd.crc as crc
    img, host, offs, lens, crc0 = zipf_image
    n = len(lens)
    rng = np.random.default_rng(78)
    split_idx = np.nonzero(lens > SEG)[0]
    whole_idx = np.nonzero(lens <= SEG)[0]
    wrong = np.sort(np.concatenate([rng.choice(split_idx, 400, replace=False),
                                    rng.choice(whole_idx, 600, replace=False)]))
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, crc0
    d["aux"][wrong] ^= (1 << rng.integers(0, 32, wrong.size)).astype(np.uint32)
    d_v = crc.DeviceBuffer(sctx, d.nbytes).upload(d)
    d_ok = crc.DeviceBuffer(sctx, n)
    d_c = crc.DeviceBuffer(sctx, 4 * n)
    d_nb = crc.DeviceBuffer(sctx, 4)
    try:
        for rep in range(2):  # twice on one stream: the slot and the plan are reused
            d_ok.zero()
            d_nb.zero()
            sctx.verify_device(d_v, n, img, d_c, d_ok, d_nb)
            st = sctx.split_stats()
            assert st["used"] > 0 and _tickets(st["units"]) >= 16 * st["grid"] * 16, st
            assert int(d_nb.download(np.uint32)[0]) == 1000, rep
            ok = d_ok.download(np.uint8, n)
            assert np.array_equal(np.nonzero(ok == 0)[0], wrong) and int((ok == 1).sum()) == n - 1000, rep
            assert np.array_equal(d_c.download(np.uint32, n), crc0), rep
    finally:
        for b in (d_v, d_ok, d_c, d_nb):
            b.free()


def test_split_launches_on_two_streams_overlap_and_agree(sctx, zipf_image):
    """Split launches of one context queued on two of its streams at once, each
    stream's scheduler slot with its own plan (no launch waits on the other
    stream's plan any more): every launch's CRCs exact."""
    import tfs_amd.crc as crc
    img, host, offs, lens, crc0 = zipf_image
    n = len(lens)
    half = n // 2
    parts = [(0, half), (half, n)]
    s1, s2 = sctx.stream_create(), sctx.stream_create()
    bufs = []
    try:
        outs = []
        for (a, b), s in zip(parts + parts, [s1, s2, s2, s1]):
            d = np.zeros(b - a, crc.DESC_DTYPE)
            d["offset"], d["len"] = offs[a:b], lens[a:b]
            d_d = crc.DeviceBuffer(sctx, d.nbytes).upload(d)
            d_o = crc.DeviceBuffer(sctx, 4 * (b - a))
            bufs += [d_d, d_o]
            sctx.batch_device(d_d, b - a, img, d_o, stream=s)
            outs.append((a, b, d_o))
        sctx.stream_sync(s1)
        sctx.stream_sync(s2)
        for a, b, d_o in outs:
            assert np.array_equal(d_o.download(np.uint32, b - a), crc0[a:b]), (a, b)
    finally:
        for x in bufs:
            x.free()
        sctx.stream_destroy(s1)
        sctx.stream_destroy(s2)
