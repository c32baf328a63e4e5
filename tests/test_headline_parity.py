"""The headline's own launch under parity: the product
schedule takes chunked tickets (CF = 4 files per ticket, the last n >> 3 one by
one) only when a launch has >= 16 files per wave (kDynMinPerWave), i.e. >= 65,536
files on 4,096 waves; with 64 KiB payloads every file is 65 stripes, so the
PF-stripe ring and the cross-file prefetch run under chunked tickets.

- 320 blocks x 1,024 x 64 KiB FileInfo-headed records (327,680 files, 21.5 GB
  on the device): the configs[1] verify launch with 1,000 wrong expectations
  (n_bad == 1,000, verdict 0 at exactly those files), every 8th block checked
  in full against the oracle, and the record-kernel verify (FileInfo checks) of
  the same image with 1,000 corrupted payloads;
- >= 300 k files of 1-16 KiB at arbitrary alignment with seeds (compute form);
- >= 300 k records of 1-4 KiB payload compacted and verified on read (jobs
  forms), byte-exact against the oracle's real_compact.

References: Func::crc src/common/func.cpp:426-435; verify sync_backup.cpp:345-435;
real_compact src/dataserver/task.cpp:753-798.
"""

import numpy as np
import pytest

from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

FILE = 65536
REC = FILE + 36
PER_BLOCK = 1024
THREADS = 16


def _oracle_mt(oracle, host, offs, lens, seeds=None):
    import tfs_amd.crc as crc
    d = np.zeros(len(offs), crc.DESC_DTYPE)
    d["offset"], d["len"] = offs, lens
    d["aux"] = 0 if seeds is None else seeds
    out = np.zeros(len(offs), np.uint32)
    assert oracle.oracle_crc_batch_mt(d.ctypes.data, len(offs), host.ctypes.data, out.ctypes.data, THREADS) == 0
    return out


@pytest.fixture(scope="module")
def headline_image(gpu_ctx):
    """320 resident blocks of the configs[1] layout, written as the bench writes them."""
    import tfs_amd.crc as crc
    ctx = gpu_ctx
    nblocks = 320
    n = nblocks * PER_BLOCK
    total = n * REC
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0xA11CE, 0)
    rec_off = np.arange(n, dtype=np.uint64) * REC
    desc = np.zeros(n, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = rec_off + 36, FILE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    ctx.batch_device(d_desc, n, img, d_crc)
    d_roff = crc.DeviceBuffer(ctx, rec_off.nbytes).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * n).upload(np.full(n, FILE, np.uint32))
    ctx.write_headers_device(img, d_roff, d_len, d_crc, 1, n)
    ctx.sync()
    expected = d_crc.download(np.uint32)
    for b in (d_desc, d_roff, d_len, d_crc):
        b.free()
    yield img, nblocks, n, total, desc, expected
    img.free()


def test_headline_launch_takes_the_chunked_path(gpu_ctx, headline_image):
    img, nblocks, n, total, desc, expected = headline_image
    waves = gpu_ctx.throughput_grid() * 16
    # the whole chip (256 CUs x 16 waves), or the chip less the 16 CUs of a resident
    # kernel that ran in this process within the last few ms (throughput_cap)
    assert waves in (4096, 4096 - 16 * 16), waves
    assert n // waves >= 16  # kDynMinPerWave: chunked tickets (FileCursor::init)


def test_headline_verify_wrong_expectations_and_oracle_blocks(gpu_ctx, oracle, headline_image):
    import tfs_amd.crc as crc
    img, nblocks, n, total, desc, expected = headline_image
    blk = PER_BLOCK * REC
    # every 8th block in full against the oracle (the device's own bytes)
    boffs = np.arange(PER_BLOCK, dtype=np.uint64) * REC + 36
    for b in range(0, nblocks, 8):
        host = img.download(np.uint8, blk, b * blk)
        got = _oracle_mt(oracle, host, boffs, np.full(PER_BLOCK, FILE))
        assert (got == expected[b * PER_BLOCK:(b + 1) * PER_BLOCK]).all(), b
        # the FileInfo headers the write path stored carry the same crc_
        fi = host.reshape(PER_BLOCK, REC)[:, :36].copy().view(crc.FILEINFO_DTYPE).reshape(-1)
        assert (fi["crc_"] == got).all() and (fi["size_"] == REC).all(), b
        assert (fi["id_"] == 1 + b * PER_BLOCK + np.arange(PER_BLOCK)).all(), b
    rng = np.random.default_rng(2024)
    bad = np.sort(rng.choice(n, 1000, replace=False))
    d = desc.copy()
    d["aux"] = expected
    d["aux"][bad] ^= (1 << rng.integers(0, 32, bad.size)).astype(np.uint32)
    d_v = crc.DeviceBuffer(gpu_ctx, d.nbytes).upload(d)
    d_ok = crc.DeviceBuffer(gpu_ctx, n)
    d_c = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_nb = crc.DeviceBuffer(gpu_ctx, 4)
    try:
        for rep in range(2):  # twice on the same stream: the slot is left clean for the next launch
            d_ok.zero()
            d_nb.zero()
            gpu_ctx.verify_device(d_v, n, img, d_c, d_ok, d_nb)
            gpu_ctx.sync()
            assert int(d_nb.download(np.uint32)[0]) == 1000, rep
            ok = d_ok.download(np.uint8, n)
            assert (np.nonzero(ok == 0)[0] == bad).all() and int((ok == 1).sum()) == n - 1000, rep
            assert (d_c.download(np.uint32, n) == expected).all(), rep
    finally:
        for b in (d_v, d_ok, d_c, d_nb):
            b.free()


def test_headline_record_verify_with_corrupted_payloads(gpu_ctx, oracle, headline_image):
    """The record kernel's verify form (FileInfo id/size checks + re-CRC, jobs
    layout) over the same 327,680 records, chunked tickets, 1,000 payloads with
    one flipped bit: status -1010 at exactly those, 0 elsewhere; the CRCs of the
    corrupted files equal the oracle's over the corrupted bytes."""
    import tfs_amd.crc as crc
    img, nblocks, n, total, desc, expected = headline_image
    rng = np.random.default_rng(2025)
    bad = np.sort(rng.choice(n, 1000, replace=False))
    pos = rng.integers(0, FILE, bad.size)
    where = bad.astype(np.uint64) * REC + 36 + pos.astype(np.uint64)
    orig = np.array([int(img.download(np.uint8, 1, int(w))[0]) for w in where], np.uint8)
    flip = (1 << rng.integers(0, 8, bad.size)).astype(np.uint8)
    jobs = np.zeros(n, crc.COMPACT_JOB_DTYPE)
    jobs["src_offset"] = np.arange(n, dtype=np.uint64) * REC
    jobs["file_id"] = 1 + np.arange(n, dtype=np.uint64)
    jobs["size"] = REC
    d_j = crc.DeviceBuffer(gpu_ctx, jobs.nbytes).upload(jobs)
    d_st = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_c = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_nb = crc.DeviceBuffer(gpu_ctx, 4)
    try:
        for w, o, f in zip(where, orig, flip):
            img.upload(np.array([o ^ f], np.uint8), int(w))
        d_nb.zero()
        gpu_ctx.blocks_verify_device(img, total, d_j, n, d_c, d_st, d_nb)
        gpu_ctx.sync()
        st = d_st.download(np.int32, n)
        assert int(d_nb.download(np.uint32)[0]) == 1000
        assert (np.nonzero(st)[0] == bad).all() and (st[bad] == -1010).all()
        c = d_c.download(np.uint32, n)
        good = np.ones(n, bool)
        good[bad] = False
        assert (c[good] == expected[good]).all()
        for i in bad[:64]:  # the corrupted files' CRCs over their corrupted bytes
            host = img.download(np.uint8, FILE, int(i) * REC + 36)
            assert int(c[i]) == int(_oracle_mt(oracle, host, [0], [FILE])[0]), i
    finally:
        for w, o in zip(where, orig):  # the module image stays clean for the other tests
            img.upload(np.array([o], np.uint8), int(w))
        for b in (d_j, d_st, d_c, d_nb):
            b.free()


def test_dynamic_path_multi_stripe_files_with_seeds(gpu_ctx, oracle):
    """>= 300 k files of 1-16 KiB (2-16 stripes each), every alignment, seeds:
    the compute form on the chunked-ticket path, against the oracle."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(2026)
    n = 300_000
    lens = rng.integers(1024, 16 * 1024 + 1, n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 64, n).astype(np.uint64))
    total = int(offs[-1] + lens[-1] + 128)
    seeds = np.where(rng.integers(0, 3, n) == 0, 0, rng.integers(0, 2**32, n)).astype(np.uint32)
    img = crc.DeviceBuffer(gpu_ctx, (total + 7) // 8 * 8)
    gpu_ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0xD1CE, 0)
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, seeds
    d_d = crc.DeviceBuffer(gpu_ctx, d.nbytes).upload(d)
    d_out = crc.DeviceBuffer(gpu_ctx, 4 * n)
    try:
        assert n // (gpu_ctx.throughput_grid() * 16) >= 16
        gpu_ctx.batch_device(d_d, n, img, d_out)
        gpu_ctx.sync()
        got = d_out.download(np.uint32, n)
        host = img.download(np.uint8, total)
        exp = _oracle_mt(oracle, host, offs, lens, seeds)
        badi = np.nonzero(got != exp)[0]
        assert badi.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16) for i in badi[:10]]
    finally:
        for b in (img, d_d, d_out):
            b.free()


def test_dynamic_path_jobs_compact_and_verify_1k_records(gpu_ctx, oracle):
    """>= 300 k records of 1-4 KiB payload, every fourth deleted, compacted in one
    tfs_compact_jobs_device launch and verified on read in one
    tfs_blocks_verify_device launch: byte-exact against the oracle's real_compact,
    CRCs and statuses exact."""
    import tfs_amd.crc as crc
    from test_gpu_parity import _oracle_compact
    rng = np.random.default_rng(2027)
    n = 320_000
    sizes = rng.integers(1024, 4097, n)
    recs = sizes + 36
    offs = np.concatenate([[0], np.cumsum(recs)[:-1]]).astype(np.int64)
    img = synth_bytes(2028, int(recs.sum()) + 256)
    c = _oracle_mt(oracle, img, offs + 36, sizes)
    fi = np.zeros(n, crc.FILEINFO_DTYPE)
    fi["id_"] = 5000 + np.arange(n)
    fi["offset_"] = offs
    fi["size_"] = fi["usize_"] = recs
    fi["crc_"] = c
    img[offs[:, None] + np.arange(36)[None, :]] = fi.view(np.uint8).reshape(n, 36)
    metas = np.zeros(n, crc.META_DTYPE)
    metas["file_id"], metas["offset"], metas["size"] = 5000 + np.arange(n), offs, recs
    fl = np.zeros(n, np.int32)
    fl[2::4] = 1
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    live = np.nonzero(fl == 0)[0]
    assert live.size >= 240_000
    j = np.zeros(live.size, crc.COMPACT_JOB_DTYPE)
    j["src_offset"], j["dest_offset"] = metas["offset"][live], doff[live]
    j["file_id"], j["size"], j["new_offset"] = metas["file_id"][live], metas["size"][live], doff[live]
    d_src = crc.DeviceBuffer(gpu_ctx, img.size).upload(img)
    d_j = crc.DeviceBuffer(gpu_ctx, j.nbytes).upload(j)
    d_dst = crc.DeviceBuffer(gpu_ctx, odest.size + 64)
    d_st = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_c = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_nb = crc.DeviceBuffer(gpu_ctx, 4)
    try:
        d_dst.zero()
        d_nb.zero()
        gpu_ctx.compact_jobs_device(d_src, img.size, d_j, live.size, d_dst, d_c, d_st, d_nb)
        gpu_ctx.sync()
        assert int(d_nb.download(np.uint32)[0]) == 0 and (d_st.download(np.int32, live.size) == 0).all()
        assert (d_c.download(np.uint32, live.size) == c[live]).all()
        assert (d_dst.download(np.uint8, odest.size) == odest).all()
        jv = np.zeros(n, crc.COMPACT_JOB_DTYPE)
        jv["src_offset"], jv["file_id"], jv["size"] = metas["offset"], metas["file_id"], metas["size"]
        jv["file_id"][7] += 1        # FileInfo id mismatch (-8016)
        jv["size"][11] += 1          # size mismatch (-8038)
        d_jv = crc.DeviceBuffer(gpu_ctx, jv.nbytes).upload(jv)
        d_nb.zero()
        gpu_ctx.blocks_verify_device(d_src, img.size, d_jv, n, d_c, d_st, d_nb)
        gpu_ctx.sync()
        st = d_st.download(np.int32, n)
        assert st[7] == -8016 and st[11] == -8038 and int(np.count_nonzero(st)) == 2
        assert int(d_nb.download(np.uint32)[0]) == 2
        cc = d_c.download(np.uint32, n)
        keep = np.ones(n, bool)
        keep[[7, 11]] = False
        assert (cc[keep] == c[keep]).all()
        d_jv.free()
    finally:
        for b in (d_src, d_j, d_dst, d_st, d_c, d_nb):
            b.free()
