"""GPU parity: the HIP path (through the C ABI) vs the oracle and the golden
vectors.  Integer/byte work, so the bar is bit-exact everywhere."""
import numpy as np
import pytest

from conftest import ocrc, vector_input
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _pack(items, align_pad=7):
    """items: list of bytes -> (buffer, offsets) with odd gaps between payloads."""
    offs, chunks, o = [], [], 0
    for i, d in enumerate(items):
        gap = (i * 5 + 3) % align_pad
        chunks.append(bytes(gap))
        o += gap
        offs.append(o)
        chunks.append(d)
        o += len(d)
    chunks.append(bytes(16))
    return np.frombuffer(b"".join(chunks), np.uint8), offs


def test_golden_vectors_gpu(gpu_ctx, golden):
    vs = golden["vectors"]
    datas = [vector_input(v) for v in vs]
    lens = [max(v.get("len_arg", len(d)), 0) for v, d in zip(vs, datas)]
    buf, offs = _pack(datas)
    got = gpu_ctx.batch(buf, offs, lens, [v["seed"] for v in vs])
    for v, g in zip(vs, got):
        assert int(g) == v["expected"], v["name"]


def test_continuation_and_datafile_gpu(gpu_ctx, golden):
    for v in golden["continuation"]:
        d = vector_input(v)
        cut = v["cut"]
        buf = np.frombuffer(d, np.uint8)
        c1 = gpu_ctx.batch(buf, [0], [cut], [v["seed"]])[0]
        assert int(c1) == v["expected_first"], v["name"]
        c2 = gpu_ctx.batch(buf, [cut], [len(d) - cut], [int(c1)])[0]
        assert int(c2) == v["expected"], v["name"]
    for v in golden["datafile_big"]:
        assert gpu_ctx.datafile_get_crc(vector_input(v)) == v["expected"], v["name"]


def test_scalar_func_crc_kats():
    import tfs_amd.crc as crc
    assert crc.func_crc(0, b"123456789") == 0x2DFD2D88
    assert crc.func_crc(0xFFFFFFFF, b"123456789") ^ 0xFFFFFFFF == 0xCBF43926
    assert crc.func_crc(0x4E534654, b"123456789") == 0xCADE6EAE
    assert crc.func_crc(0, b"\x80") == 0xEDB88320
    assert crc.func_crc(0x1234, b"") == 0x1234
    assert crc.func_crc(7, b"abcde", -5) == 7
    assert crc.func_crc(0, b"1" + bytes(31)) == 0xD631B691


@pytest.mark.parametrize("seed_mode", ["zero", "random"])
def test_all_small_lengths_and_alignments(gpu_ctx, oracle, seed_mode):
    rng = np.random.default_rng(11 if seed_mode == "zero" else 12)
    lens = list(range(0, 600)) + [int(x) for x in rng.integers(600, 20000, 150)]
    buf = synth_bytes(99, sum(lens) + 32 * len(lens) + 64)
    raw = buf.tobytes()
    offs, o = [], 0
    for i, n in enumerate(lens):
        o += i % 16 + 1
        offs.append(o)
        o += n
    seeds = [0] * len(lens) if seed_mode == "zero" else [int(x) for x in rng.integers(0, 2**32, len(lens))]
    got = gpu_ctx.batch(buf, offs, lens, seeds)
    for i, n in enumerate(lens):
        assert int(got[i]) == ocrc(oracle, seeds[i], raw[offs[i]:offs[i] + n]), (i, n, offs[i] % 16)


def test_large_sizes(gpu_ctx, oracle):
    sizes = [65535, 65536, 65537, 65536 * 64 - 5, (1 << 20) + 1, 3 * (1 << 20) + 17, 9 * (1 << 20) + 3]
    for k, n in enumerate(sizes):
        for off in (0, 4, 13):
            buf = synth_bytes(300 + k, n + off + 8)
            raw = buf.tobytes()
            s = [0, 0x4E534654, 0xFFFFFFFF][k % 3]
            got = gpu_ctx.batch(buf, [off], [n], [s])[0]
            assert int(got) == ocrc(oracle, s, raw[off:off + n]), (n, off)


def test_verify_detects_every_single_byte_corruption(gpu_ctx, oracle):
    n, ln = 96, 65536
    stride = ln + 36
    buf = synth_bytes(5, n * stride + 64)
    raw = bytearray(buf.tobytes())
    offs = [36 + i * stride for i in range(n)]
    exp = [ocrc(oracle, 0, raw[o:o + ln]) for o in offs]
    rng = np.random.default_rng(3)
    bad_files = sorted(rng.choice(n, 17, replace=False).tolist())
    for f in bad_files:
        pos = offs[f] + int(rng.integers(0, ln))
        raw[pos] ^= 1 << int(rng.integers(0, 8))
    crc, ok, nbad, rc = gpu_ctx.verify(np.frombuffer(bytes(raw), np.uint8), offs, [ln] * n, exp)
    assert nbad == len(bad_files) and rc == -1010
    assert [i for i in range(n) if not ok[i]] == bad_files
    for i in range(n):
        assert int(crc[i]) == ocrc(oracle, 0, raw[offs[i]:offs[i] + ln])


def test_async_submit_wait(gpu_ctx, oracle):
    hs, exps = [], []
    for k in range(3):
        buf = synth_bytes(700 + k, 10 * 4096 + 8)
        offs = [i * 4096 + 4 for i in range(10)]
        exp = [ocrc(oracle, 0, buf[o:o + 4000].tobytes()) for o in offs]
        if k == 1:
            exp[4] ^= 0x10
        hs.append(gpu_ctx.submit_verify(buf, offs, [4000] * 10, exp))
    for k, h in enumerate(hs):
        crc, ok, nbad, rc = gpu_ctx.wait(h)
        assert nbad == (1 if k == 1 else 0)


def test_device_resident(gpu_ctx, oracle):
    import tfs_amd.crc as crc
    n, ln = 512, 65536
    stride = ln + 36
    nbytes = (n * stride + 4095) // 4096 * 4096
    img = crc.DeviceBuffer(gpu_ctx, nbytes)
    gpu_ctx.synth_fill_device(img, nbytes, 1234, 0)
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"] = 36 + np.arange(n) * stride
    d["len"] = ln
    dd = crc.DeviceBuffer(gpu_ctx, d.nbytes).upload(d)
    out = crc.DeviceBuffer(gpu_ctx, 4 * n)
    gpu_ctx.batch_device(dd, n, img, out)
    gpu_ctx.sync()
    host = synth_bytes(1234, nbytes)
    assert (img.download() == host).all()
    got = out.download(np.uint32)
    for i in range(0, n, 37):
        o = int(d["offset"][i])
        assert int(got[i]) == ocrc(oracle, 0, host[o:o + ln].tobytes())
    # verify on device against the computed CRCs, with two corrupted expectations
    v = d.copy()
    v["aux"] = got
    v["aux"][[3, 300]] ^= 1
    vd = crc.DeviceBuffer(gpu_ctx, v.nbytes).upload(v)
    okd = crc.DeviceBuffer(gpu_ctx, n)
    nb = crc.DeviceBuffer(gpu_ctx, 4)
    nb.zero()
    gpu_ctx.verify_device(vd, n, img, None, okd, nb)
    gpu_ctx.sync()
    assert int(nb.download(np.uint32)[0]) == 2
    assert sorted(np.nonzero(okd.download() == 0)[0].tolist()) == [3, 300]


def _block_image(oracle, sizes, seed=21):
    """Pack FileInfo|payload records like LogicBlock::close_write_file does."""
    import tfs_amd.crc as crc
    total = sum(36 + s for s in sizes)
    img = np.zeros(total + 64, np.uint8)
    metas = np.zeros(len(sizes), crc.META_DTYPE)
    o = 0
    for i, s in enumerate(sizes):
        pay = synth_bytes(seed * 1000 + i, s)
        fi = np.zeros(1, crc.FILEINFO_DTYPE)
        fi["id_"] = 1000 + i
        fi["offset_"] = o
        fi["size_"] = s + 36
        fi["usize_"] = s + 36
        fi["crc_"] = ocrc(oracle, 0, pay.tobytes())
        img[o:o + 36] = fi.view(np.uint8)
        img[o + 36:o + 36 + s] = pay
        metas[i] = (1000 + i, o, s + 36)
        o += 36 + s
    return img, metas


def test_block_verify_statuses(gpu_ctx, oracle):
    sizes = [65536] * 20 + [1, 100, 4097, 70001]
    img, metas = _block_image(oracle, sizes)
    crc_, st, nbad, rc = gpu_ctx.block_verify(img, metas)
    assert nbad == 0 and (st == 0).all()
    img[int(metas[5]["offset"]) + 36 + 777] ^= 0x40            # payload corruption
    metas2 = metas.copy()
    metas2[7]["file_id"] = 999999                               # header id mismatch
    img[int(metas[9]["offset"]) + 12] ^= 0x01                   # FileInfo.size_ mismatch
    metas2[11]["size"] = 36                                     # too short
    crc_, st, nbad, rc = gpu_ctx.block_verify(img, metas2)
    assert rc == -1010 and nbad == 4
    assert st[5] == -1010 and st[7] == -8016 and st[9] == -8038 and st[11] == -8034
    for i in (0, 21, 23):
        o = int(metas[i]["offset"])
        code = oracle.oracle_verify_file(img.ctypes.data, img.size, o, int(metas[i]["size"]), None)
        assert code == st[i] == 0


def test_block_compact_matches_oracle(gpu_ctx, oracle):
    rng = np.random.default_rng(8)
    sizes = [65536] * 30 + [int(x) for x in rng.integers(1, 9000, 30)]
    img, metas = _block_image(oracle, sizes, seed=33)
    flags = np.zeros(len(sizes), np.int32)
    flags[::2] |= 1                 # delete every even file (test_logic_block_and_compact.cpp:946-975)
    flags[1::6] |= 2                # and invalidate some
    flags[3::10] |= 4               # concealed files survive
    img[int(metas[5]["offset"]) + 40] ^= 1   # a live file with a bad payload
    dest, dmetas, ok, rc = gpu_ctx.block_compact(img, metas, flags)
    n = len(sizes)
    mo = metas["offset"].astype(np.int64)
    ms = metas["size"].astype(np.int32)
    odest = np.zeros(dest.size + 64, np.uint8)
    doff = np.zeros(n, np.int64)
    dsz = np.zeros(n, np.int32)
    ook = np.zeros(n, np.uint8)
    w = oracle.oracle_compact(img.ctypes.data, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data, n,
                              odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
    assert w == dest.size
    assert (odest[:w] == dest).all()
    assert (ook == ok).all()
    assert rc == -1010 and ok[5] == 0
    live = [i for i in range(n) if not flags[i] & 3]
    assert [int(x) for x in dmetas["file_id"]] == [int(metas[i]["file_id"]) for i in live]
    assert [int(x) for x in dmetas["offset"]] == [int(doff[i]) for i in live]


def _oracle_compact(oracle, img, metas, flags):
    n = len(metas)
    mo = metas["offset"].astype(np.int64)
    ms = metas["size"].astype(np.int32)
    odest = np.zeros(int(ms.sum()) + 64, np.uint8)
    doff = np.zeros(n, np.int64)
    dsz = np.zeros(n, np.int32)
    ook = np.zeros(n, np.uint8)
    w = oracle.oracle_compact(img.ctypes.data, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data, n,
                              odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
    return odest[:w], doff, ook


def test_compact_fused_every_shift_class(gpu_ctx, oracle):
    """The fused compaction kernel stores payload registers at dst = src + delta:
    delta = 0 mod 16 (nt 16-byte stores), 4/8/12 mod 16 (dword stores) and
    not 0 mod 4 (byte-copy fallback) -- all byte-identical to the oracle's
    real_compact restatement, with payloads from 1 byte to several stripes."""
    rng = np.random.default_rng(91)
    sizes, flags = [], []
    for k in range(160):
        sizes.append(int(rng.choice([1, 3, 17, 31, 32, 33, 100, 1023, 1024, 1025, 2049, 5000, 65536, 70001])))
        # deleting a record of s bytes shifts every later record by s + 36 (mod 16: k % 16)
        flags.append(1 if k % 3 == 1 else 0)
        if flags[-1]:
            sizes[-1] = 16 + (k % 16 - 36) % 16
    img, metas = _block_image(oracle, sizes, seed=71)
    fl = np.array(flags, np.int32)
    img[int(metas[10]["offset"]) + 36 + 3] ^= 0x80
    dest, dmetas, ok, rc = gpu_ctx.block_compact(img, metas, fl)
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    assert dest.size == odest.size and (dest == odest).all()
    assert (ok == ook).all()
    live = [i for i in range(len(sizes)) if not fl[i]]
    deltas = {(int(doff[i]) - int(metas[i]["offset"])) % 16 for i in live}
    assert {0, 4, 8, 12} <= deltas and deltas - {0, 4, 8, 12}  # every class exercised


def test_block_compact_device_matches_oracle(gpu_ctx, oracle):
    import tfs_amd.crc as crc
    rng = np.random.default_rng(92)
    sizes = [65536] * 50 + [int(x) for x in rng.integers(1, 30000, 50)]
    img, metas = _block_image(oracle, sizes, seed=72)
    fl = np.zeros(len(sizes), np.int32)
    fl[::3] = 1
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    live = np.nonzero((fl & 3) == 0)[0]
    lm = np.ascontiguousarray(metas[live])
    lf = np.ascontiguousarray(fl[live])
    ld = np.concatenate([[0], np.cumsum(lm["size"].astype(np.int64))[:-1]]).astype(np.int64)
    n = len(live)
    d_src = crc.DeviceBuffer(gpu_ctx, img.size).upload(img)
    d_m = crc.DeviceBuffer(gpu_ctx, lm.nbytes).upload(lm)
    d_f = crc.DeviceBuffer(gpu_ctx, lf.nbytes).upload(lf)
    d_o = crc.DeviceBuffer(gpu_ctx, ld.nbytes).upload(ld)
    d_dst = crc.DeviceBuffer(gpu_ctx, odest.size + 64)
    d_crc = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_st = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_bad = crc.DeviceBuffer(gpu_ctx, 4)
    d_bad.zero()
    gpu_ctx.block_compact_device(d_src, img.size, d_m, d_f, d_o, n, d_dst, d_crc, d_st, d_bad)
    gpu_ctx.sync()
    assert (d_dst.download(np.uint8, odest.size) == odest).all()
    assert (d_st.download(np.int32, n) == 0).all() and int(d_bad.download(np.uint32, 1)[0]) == 0
    assert (ook[live] == 1).all()


def test_compact_jobs_device_many_blocks(gpu_ctx, oracle):
    """tfs_compact_jobs_device: several blocks' live records in one launch,
    each block packed into its own destination region; equals the oracle's
    real_compact of every block."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(93)
    blocks, jobs, expect = [], [], []
    src_base = dst_base = 0
    for b in range(5):
        sizes = [65536] * 12 + [int(x) for x in rng.integers(1, 12000, 20)]
        img, metas = _block_image(oracle, sizes, seed=80 + b)
        fl = np.zeros(len(sizes), np.int32)
        fl[b % 3::3] = 1
        odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
        for i in np.nonzero((fl & 3) == 0)[0]:
            jobs.append((src_base + int(metas[i]["offset"]), dst_base + int(doff[i]), int(metas[i]["file_id"]),
                         int(metas[i]["size"]), int(fl[i]), int(doff[i]), 0))
        blocks.append(img[:int(metas["size"].astype(np.int64).sum())])
        expect.append((dst_base, odest))
        src_base += blocks[-1].size
        dst_base += odest.size + (b * 7) % 16   # destination blocks at assorted alignments
    src = np.concatenate(blocks)
    j = np.array(jobs, dtype=crc.COMPACT_JOB_DTYPE)
    rng.shuffle(j)   # any order
    d_src = crc.DeviceBuffer(gpu_ctx, src.size + 64).upload(src)
    d_j = crc.DeviceBuffer(gpu_ctx, j.nbytes).upload(j)
    d_dst = crc.DeviceBuffer(gpu_ctx, dst_base + 64)
    d_dst.zero()
    d_st = crc.DeviceBuffer(gpu_ctx, 4 * len(j))
    d_bad = crc.DeviceBuffer(gpu_ctx, 4)
    d_bad.zero()
    gpu_ctx.compact_jobs_device(d_src, src.size, d_j, len(j), d_dst, None, d_st, d_bad)
    gpu_ctx.sync()
    out = d_dst.download(np.uint8, dst_base)
    for base, od in expect:
        assert (out[base:base + od.size] == od).all()
    assert int(d_bad.download(np.uint32, 1)[0]) == 0


def _stripe_edge_cases(run, count=24):
    """(offset, len) pairs where the payload starts inside the last dword of
    stripe 0, so the high seed bytes land in stripe 1 (lane 0)."""
    S = 64 * run
    out = []
    for st in range(16, 64):
        if st % 4 == 0:
            continue
        for ln in list(range(40, 200)) + list(range(S - 40, 4 * S + 40, 3)):
            end = st + ln
            A, B16 = st & ~3, end & ~15
            E = (B16 + 127) & ~127 if run == 16 else B16   # the kernel's stripe anchor
            body = E - A
            ns = (body + S - 1) // S
            if ln >= 32 and A + 4 == E - ns * S + S:
                out.append((st, ln))
        if len(out) >= count:
            break
    return out[:count]


@pytest.mark.parametrize("variant", [0, 20, 50])
def test_kernel_variants_parity(oracle, variant, monkeypatch):
    """The product, the latency form forced on every batch (TFS_CRC_VARIANT 20) and
    one file per ticket (50) are bit-exact, including the stripe-0 seed edge."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(variant))
    ctx = crc.Context(0)
    try:
        rng = np.random.default_rng(100 + variant)
        items = []
        for run in (16, 32, 64):
            items += _stripe_edge_cases(run)
        items += [(int(rng.integers(0, 16)), int(n)) for n in rng.integers(1, 300000, 40)]
        items += [(3, 65536), (0, 65536), (36, 65536), (1, 31), (2, 32), (5, 0)]
        buf = synth_bytes(4242 + variant, max(o + n for o, n in items) + 64)
        raw = buf.tobytes()
        seeds = [int(x) for x in rng.integers(0, 2**32, len(items))]
        got = ctx.batch(buf, [o for o, _ in items], [n for _, n in items], seeds)
        for (o, n), sd, g in zip(items, seeds, got):
            assert int(g) == ocrc(oracle, sd, raw[o:o + n]), (variant, o, n)
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [0, 20, 50])
def test_cross_file_pipeline_many_files(oracle, variant, monkeypatch):
    """> 4096 files so every wave runs a sequence of files of mixed geometry
    (tiny / single-stripe / multi-stripe, any alignment, any seed): exercises
    the next-file prefetch of the persistent kernel."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(variant))
    ctx = crc.Context(0)
    try:
        rng = np.random.default_rng(777 + variant)
        n = 3 * 4096 + 517
        kind = rng.integers(0, 4, n)
        lens = np.where(kind == 0, rng.integers(0, 32, n),
                        np.where(kind == 1, rng.integers(32, 1100, n),
                                 np.where(kind == 2, rng.integers(1100, 9000, n), rng.integers(9000, 70000, n))))
        gaps = rng.integers(0, 16, n)
        offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1]])).astype(np.uint64)
        total = int(offs[-1] + lens[-1] + 64)
        buf = synth_bytes(31337 + variant, total)
        seeds = np.where(rng.integers(0, 2, n) == 0, 0, rng.integers(0, 2**32, n)).astype(np.uint32)
        got = ctx.batch(buf, offs, lens, seeds)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"], d["len"], d["aux"] = offs, lens, seeds
        exp = np.zeros(n, np.uint32)
        oracle.oracle_crc_batch(d.ctypes.data, n, buf.ctypes.data, exp.ctypes.data)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16, int(seeds[i])) for i in bad[:10]]
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [0, 50])
def test_dynamic_tickets_million_files(oracle, variant, monkeypatch):
    """> 16 files (or chunks of CF files, the product) per wave, so the launch
    takes the dynamic-ticket path with stealing across the eight groups: 1 M short
    files of every length class below 300 bytes, any alignment and seed."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(variant))
    ctx = crc.Context(0)
    try:
        rng = np.random.default_rng(4040 + variant)
        n = (1 << 20) + 777
        lens = rng.integers(0, 300, n)
        offs = np.cumsum(rng.integers(0, 8, n) + np.concatenate([[0], lens[:-1]])).astype(np.uint64)
        buf = synth_bytes(9090 + variant, int(offs[-1] + lens[-1] + 64))
        seeds = np.where(rng.integers(0, 2, n) == 0, 0, rng.integers(0, 2**32, n)).astype(np.uint32)
        got = ctx.batch(buf, offs, lens, seeds)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"], d["len"], d["aux"] = offs, lens, seeds
        exp = np.zeros(n, np.uint32)
        oracle.oracle_crc_batch(d.ctypes.data, n, buf.ctypes.data, exp.ctypes.data)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (variant, bad.size, [(int(i), int(lens[i])) for i in bad[:10]])
    finally:
        ctx.close()


def test_blocks_compact_pipelined_matches_oracle(gpu_ctx, oracle):
    """Many blocks through the 3-stream compaction pipeline; every block's output
    equals the oracle's real_compact restatement; pinned and pageable images."""
    import ctypes
    import tfs_amd.crc as crc
    rng = np.random.default_rng(44)
    nblk = 7
    keep = []
    jobs = (crc.BlockJob * nblk)()
    expect = []
    for b in range(nblk):
        sizes = [65536] * 40 + [int(x) for x in rng.integers(1, 20000, 25)]
        img, metas = _block_image(oracle, sizes, seed=60 + b)
        flags = np.zeros(len(sizes), np.int32)
        flags[b % 2::2] |= 1
        flags[1::3] |= 2 if b % 3 == 0 else 0
        if b == 4:
            img[int(metas[3]["offset"]) + 50] ^= 4   # one corrupted live file (flags[3] live for b even)
        if b % 2 == 0:
            pin = crc.PinnedBuffer(gpu_ctx, img.size)
            pin.array[:] = img
            src = pin
            src_ptr, src_arr = pin.ptr, pin.array
        else:
            src, src_ptr, src_arr = img, img.ctypes.data, img
        cap = int(metas["size"].sum()) + 64
        dest = np.zeros(cap, np.uint8)
        dm = np.zeros(len(sizes), crc.META_DTYPE)
        ok = np.zeros(len(sizes), np.uint8)
        keep.append((src, img, metas, flags, dest, dm, ok))
        j = jobs[b]
        j.src_image, j.src_len, j.metas, j.flags, j.n = src_ptr, img.size, metas.ctypes.data, flags.ctypes.data, len(sizes)
        j.dest_image, j.dest_cap, j.dest_metas, j.crc_ok = dest.ctypes.data, cap, dm.ctypes.data, ok.ctypes.data
        n = len(sizes)
        mo = metas["offset"].astype(np.int64)
        ms = metas["size"].astype(np.int32)
        odest = np.zeros(cap, np.uint8)
        doff = np.zeros(n, np.int64)
        dsz = np.zeros(n, np.int32)
        ook = np.zeros(n, np.uint8)
        w = oracle.oracle_compact(src_arr.ctypes.data, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data, n,
                                  odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
        expect.append((w, odest[:w].copy(), ook))
    rc = gpu_ctx.blocks_compact(jobs)
    assert rc == -1010
    for b in range(nblk):
        src, img, metas, flags, dest, dm, ok = keep[b]
        w, odest, ook = expect[b]
        assert jobs[b].dest_len == w
        assert (dest[:w] == odest).all(), b
        assert (ok == ook).all(), b
        assert jobs[b].status == (-1010 if b == 4 else 0)
    for k in keep:
        if isinstance(k[0], crc.PinnedBuffer):
            k[0].free()


def test_blocks_compact_zero_copy_groups(gpu_ctx, oracle, monkeypatch):
    """tfs_blocks_compact sends runs of up to 64 page-locked blocks to the GPU as one
    multi-block record launch (round 5): 37 blocks in separate
    page-locked allocations, a pageable block in the middle (the run breaks there
    and it takes the per-block path), a block with every record deleted, records of
    every size class and destination shift, records ending exactly at their image's
    end (TFS_COMPACT_JOB_EDGE: no read past them), corrupted records in two blocks.
    Every block's bytes, new RawMeta list, crc_ok, status, dest_len and n_live equal
    the oracle's real_compact; run twice on the same context, and once more on a
    context of 8 blocks per launch (TFS_CRC_COMPACT_GROUP), where runs are cut by
    the group size too."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_COMPACT_GROUP", "8")
    ctx8 = crc.Context(0)
    monkeypatch.delenv("TFS_CRC_COMPACT_GROUP")
    rng = np.random.default_rng(4501)
    nblk = 37
    bufs, keep = [], []
    try:
        for b in range(nblk):
            if b % 5 == 0:
                sizes = [65536] * 30
            else:
                sizes = [int(x) for x in rng.choice([1, 3, 33, 100, 1023, 4096, 5001, 65536, 70001], 25)]
            img, metas = _block_image(oracle, sizes, seed=4600 + b)
            img = img[:int(metas["size"].astype(np.int64).sum())].copy()  # the last record ends the image
            flags = np.zeros(len(sizes), np.int32)
            flags[(b + 1) % 3::3] |= 1
            if b == 9:
                flags[:] = 1                                               # nothing live
            if b in (5, 30):
                live = np.nonzero(flags == 0)[0]
                k = int(live[len(live) // 2])
                img[int(metas[k]["offset"]) + 36 + int(metas[k]["size"]) // 3 - 12] ^= 0x40
            if b == 17:
                src_ptr, src_arr, srcbuf = img.ctypes.data, img, None      # pageable: breaks the run
            else:
                srcbuf = crc.PinnedBuffer(gpu_ctx, img.size)
                srcbuf.array[:] = img
                bufs.append(srcbuf)
                src_ptr, src_arr = srcbuf.ptr, srcbuf.array
            cap = int(metas["size"].astype(np.int64).sum()) + 64
            dst = crc.PinnedBuffer(gpu_ctx, cap)
            bufs.append(dst)
            odest, doff, ook = _oracle_compact(oracle, img, metas, flags)
            keep.append((src_ptr, img, metas, flags, dst, cap, odest, doff, ook))
        for rep, ctx in enumerate((gpu_ctx, gpu_ctx, ctx8)):
            jobs = (crc.BlockJob * nblk)()
            outs = []
            for b, (src_ptr, img, metas, flags, dst, cap, odest, doff, ook) in enumerate(keep):
                dst.array[:] = 0
                ok = np.full(len(metas), 7, np.uint8)
                dm = np.zeros(len(metas), crc.META_DTYPE)
                outs.append((ok, dm))
                j = jobs[b]
                j.src_image, j.src_len, j.metas, j.flags, j.n = src_ptr, img.size, metas.ctypes.data, \
                    flags.ctypes.data, len(metas)
                j.dest_image, j.dest_cap, j.dest_metas, j.crc_ok = dst.ptr, cap, dm.ctypes.data, ok.ctypes.data
            assert ctx.blocks_compact(jobs) == -1010
            for b, (src_ptr, img, metas, flags, dst, cap, odest, doff, ook) in enumerate(keep):
                ok, dm = outs[b]
                live = np.nonzero((flags & 3) == 0)[0]
                w = int(jobs[b].dest_len)
                assert w == odest.size and jobs[b].n_live == live.size, (rep, b)
                assert (dst.array[:w] == odest).all(), (rep, b)
                assert (ok == ook).all(), (rep, b)
                assert jobs[b].status == (-1010 if b in (5, 30) else 0), (rep, b)
                assert (dm["file_id"][:live.size] == metas["file_id"][live]).all(), (rep, b)
                assert (dm["offset"][:live.size] == doff[live]).all(), (rep, b)
                assert (dm["size"][:live.size] == metas["size"][live]).all(), (rep, b)
    finally:
        for p in bufs:
            p.free()
        ctx8.close()


def _pinned_group_blocks(gpu_ctx, oracle, nblk, seed, bufs):
    """nblk page-locked source/destination block pairs with their oracle results."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(seed)
    keep = []
    for b in range(nblk):
        sizes = [int(x) for x in rng.choice([1, 33, 1023, 4096, 65536, 70001], 20)]
        img, metas = _block_image(oracle, sizes, seed=seed + b)
        img = img[:int(metas["size"].astype(np.int64).sum())].copy()
        flags = np.zeros(len(sizes), np.int32)
        flags[b % 3::3] |= 1
        src = crc.PinnedBuffer(gpu_ctx, img.size)
        src.array[:] = img
        cap = int(metas["size"].astype(np.int64).sum()) + 64
        dst = crc.PinnedBuffer(gpu_ctx, cap)
        bufs += [src, dst]
        keep.append([src, img, metas, flags, dst, cap])
    return keep


def _group_jobs(keep):
    import tfs_amd.crc as crc
    jobs = (crc.BlockJob * len(keep))()
    outs = []
    for b, (src, img, metas, flags, dst, cap) in enumerate(keep):
        dst.array[:] = 0
        ok = np.full(len(metas), 7, np.uint8)
        dm = np.zeros(len(metas), crc.META_DTYPE)
        outs.append((ok, dm))
        j = jobs[b]
        j.src_image, j.src_len, j.metas, j.flags, j.n = src.ptr, img.size, metas.ctypes.data, flags.ctypes.data, \
            len(metas)
        j.dest_image, j.dest_cap, j.dest_metas, j.crc_ok = dst.ptr, cap, dm.ctypes.data, ok.ctypes.data
        j.status = 12345
    return jobs, outs


def _check_group_block(oracle, keep_b, job, out, tag):
    src, img, metas, flags, dst, cap = keep_b
    odest, doff, ook = _oracle_compact(oracle, src.array.copy(), metas, flags)
    ok, dm = out
    live = np.nonzero((flags & 3) == 0)[0]
    w = int(job.dest_len)
    assert w == odest.size and job.n_live == live.size, tag
    assert (dst.array[:w] == odest).all(), tag
    assert (ok == ook).all(), tag
    assert job.status == (0 if (ook[live] == 1).all() else -1010), tag
    assert (dm["offset"][:live.size] == doff[live]).all(), tag


def test_blocks_compact_group_failures(gpu_ctx, oracle):
    """the failure paths of a zero-copy group.  A pinned run of 12 blocks
    (more than the 8 compaction slots, so the per-job fallback reuses the slot the
    failed group held) with an out-of-range meta in block 4 and a too-small
    dest_cap in block 7: those two report TFS_EXIT_PARAMETER_ERROR with nothing
    written, every other block (one with a corrupted record) equals the oracle.
    Then a device error injected in the middle of the fallback: the blocks issued
    before it finish, it and every later block carry the device error, and the
    call returns it.  After each, a clean call on the same context is exact and
    leaves the earlier call's job array untouched (no stale slot state)."""
    import ctypes
    bufs = []
    try:
        keep = _pinned_group_blocks(gpu_ctx, oracle, 12, 7100, bufs)
        live10 = np.nonzero((keep[10][3] & 3) == 0)[0]
        k = int(live10[0])
        keep[10][0].array[int(keep[10][2][k]["offset"]) + 36 + int(keep[10][2][k]["size"]) // 2 - 20] ^= 0x08

        def run(jobs):
            return gpu_ctx.L.tfs_blocks_compact(gpu_ctx.handle, ctypes.cast(jobs, ctypes.c_void_p), len(jobs))

        # (1) parameter errors inside the group
        bad_metas = keep[4][2].copy()
        bad_metas[3]["offset"] = keep[4][1].size  # past the image
        jobs1, outs1 = _group_jobs(keep)
        jobs1[4].metas = bad_metas.ctypes.data
        jobs1[7].dest_cap = 100
        assert run(jobs1) == -1016
        for b in range(12):
            if b in (4, 7):
                assert jobs1[b].status == -1016 and jobs1[b].dest_len == 0 and jobs1[b].n_live == 0, b
            else:
                _check_group_block(oracle, keep[b], jobs1[b], outs1[b], ("param", b))
        snap1 = [(j.status, j.dest_len, j.n_live) for j in jobs1]

        jobs2, outs2 = _group_jobs(keep)
        assert run(jobs2) == -1010
        for b in range(12):
            _check_group_block(oracle, keep[b], jobs2[b], outs2[b], ("clean", b))
        assert [(j.status, j.dest_len, j.n_live) for j in jobs1] == snap1

        # (2) a device error in the per-job fallback: the group consults the fault
        # hook for jobs 0..4 before rejecting job 4, the fallback once per job.  The
        # call returns its first non-CRC error (the group's parameter error); every
        # job from the failed one on carries the device error.
        jobs3, outs3 = _group_jobs(keep)
        jobs3[4].metas = bad_metas.ctypes.data
        gpu_ctx.inject_device_error(5 + 3, 1)
        assert run(jobs3) == -1016
        for b in range(3):
            _check_group_block(oracle, keep[b], jobs3[b], outs3[b], ("dev", b))
        for b in range(3, 12):
            assert jobs3[b].status == -20001 and jobs3[b].dest_len == 0 and jobs3[b].n_live == 0, b
        snap3 = [(j.status, j.dest_len, j.n_live) for j in jobs3]

        jobs4, outs4 = _group_jobs(keep)
        assert run(jobs4) == -1010
        for b in range(12):
            _check_group_block(oracle, keep[b], jobs4[b], outs4[b], ("after", b))
        assert [(j.status, j.dest_len, j.n_live) for j in jobs3] == snap3
    finally:
        gpu_ctx.inject_device_error(0, 0)
        for p in bufs:
            p.free()


def test_blocks_compact_zero_copy_matches_oracle(gpu_ctx, oracle, monkeypatch):
    """Page-locked source and destination images: the fused kernel reads the live
    records over PCIe and writes the new block in place (no whole-block DMA).
    Records congruent mod 4 take that path; a block with arbitrary record sizes
    falls back to the DMA form.  Every block equals the oracle's real_compact
    restatement, and the DMA form (TFS_CRC_VARIANT=8) gives the same bytes."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(45)
    shapes = [
        [65536] * 48,                                                     # BASELINE records (65,572 B)
        [int(x) * 4 for x in rng.integers(1, 3000, 60)],                  # any size, multiple of 4
        [int(x) for x in rng.integers(1, 12000, 50)],                     # arbitrary: DMA fallback
        [65536] * 10 + [9 * 1024 * 1024 + 4] + [4096] * 10,              # a > 8 MiB "big file"
    ]
    monkeypatch.setenv("TFS_CRC_VARIANT", "8")
    dma_ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    bufs = []
    try:
        results = {}
        for name, ctx in (("zc", gpu_ctx), ("dma", dma_ctx)):
            jobs = (crc.BlockJob * len(shapes))()
            keep = []
            for b, sizes in enumerate(shapes):
                img, metas = _block_image(oracle, sizes, seed=90 + b)
                flags = np.zeros(len(sizes), np.int32)
                flags[(b + 1) % 2::2] |= 1
                if b == 3:
                    flags[10] = 0                                           # keep the big file
                if b == 1:
                    img[int(metas[5]["offset"]) + 40] ^= 8                  # a corrupted live file
                src = crc.PinnedBuffer(ctx, img.size)
                src.array[:] = img
                cap = int(metas["size"].astype(np.int64).sum()) + 64
                dst = crc.PinnedBuffer(ctx, cap)
                dst.array[:] = 0
                bufs += [src, dst]
                ok = np.zeros(len(sizes), np.uint8)
                dm = np.zeros(len(sizes), crc.META_DTYPE)
                keep.append((img, metas, flags, dst, ok, dm))
                j = jobs[b]
                j.src_image, j.src_len, j.metas, j.flags, j.n = src.ptr, img.size, metas.ctypes.data, \
                    flags.ctypes.data, len(sizes)
                j.dest_image, j.dest_cap, j.dest_metas, j.crc_ok = dst.ptr, cap, dm.ctypes.data, ok.ctypes.data
            rc = ctx.blocks_compact(jobs)
            assert rc == -1010
            out = []
            for b, (img, metas, flags, dst, ok, dm) in enumerate(keep):
                odest, doff, ook = _oracle_compact(oracle, img, metas, flags)
                w = int(jobs[b].dest_len)
                assert w == odest.size, (name, b)
                assert (dst.array[:w] == odest).all(), (name, b)
                assert (ok == ook).all(), (name, b)
                assert jobs[b].status == (-1010 if b == 1 else 0), (name, b)
                out.append(dst.array[:w].copy())
            results[name] = out
        for a, b in zip(results["zc"], results["dma"]):
            assert (a == b).all()
    finally:
        for p in bufs:
            p.free()
        dma_ctx.close()


def test_block_verify_zero_copy_pinned_image(gpu_ctx, oracle):
    """A page-locked block image is verified in place (zero-copy, only the named
    records cross PCIe): same CRCs and statuses as the staged pageable path,
    including out-of-range metas, which must not be read."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(46)
    sizes = [65536] * 30 + [int(x) for x in rng.integers(1, 20000, 30)]
    img, metas = _block_image(oracle, sizes, seed=47)
    img[int(metas[4]["offset"]) + 36 + 9] ^= 0x02
    live = np.ascontiguousarray(metas[1::3])                      # a fragmented block: every 3rd record
    bad_meta = np.zeros(1, crc.META_DTYPE)
    bad_meta[0] = (5, img.size - 10, 4096)                        # runs past the image
    m = np.concatenate([live, bad_meta])
    pin = crc.PinnedBuffer(gpu_ctx, img.size)
    try:
        pin.array[:] = img
        c1, s1, n1, r1 = gpu_ctx.block_verify(pin.array, m)
        c2, s2, n2, r2 = gpu_ctx.block_verify(img.copy(), m)
        assert (s1 == s2).all() and n1 == n2 and r1 == r2
        assert (c1[:-1] == c2[:-1]).all()
        assert s1[-1] == -1016 and s1[1] == -1010 and (s1[2:-1] == 0).all() and s1[0] == 0
        for i in range(len(live)):
            o, sz = int(live[i]["offset"]), int(live[i]["size"])
            assert int(c1[i]) == ocrc(oracle, 0, img[o + 36:o + sz].tobytes())
        # the same slot again with another meta list (metas, CRCs and statuses go
        # through its page-locked words: nothing of the previous call may remain)
        m2 = np.ascontiguousarray(live[::-2])
        c3, s3, n3, r3 = gpu_ctx.block_verify(pin.array, m2)
        c4, s4, n4, r4 = gpu_ctx.block_verify(img.copy(), m2)
        assert (c3 == c4).all() and (s3 == s4).all() and n3 == n4 and r3 == r4
    finally:
        pin.free()


def test_wide_pinned_batches_read_in_place(gpu_ctx, oracle, monkeypatch):
    """A page-locked batch wider than 8 MiB with more than 256 files (a block image
    read back for verify) runs as one throughput launch that reads the files, its
    descriptors and writes its verdicts in host memory (round 5): tfs_crc32_verify,
    tfs_crc32_batch and three submissions in flight give the oracle's CRCs and the
    same verdicts as the pageable path and as the staged form (TFS_CRC_VARIANT=52);
    files over 128 KiB take the split plan over host-resident descriptors."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(5252)
    n = 700
    lens = rng.integers(0, 60000, n).astype(np.uint32)
    lens[:6] = [0, 1, 3, 4, 65536, 300 * 1024 + 5]                    # one file to split
    lens[n // 2] = 1 << 20
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 9, n - 1).astype(np.uint64))
    size = int(offs[-1] + lens[-1]) + 64
    assert size > 8 << 20
    data = rng.integers(0, 256, size, dtype=np.uint8)
    exp = np.array([ocrc(oracle, 0, data[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)], np.uint32)
    bad = np.array([5, 77, n // 2, n - 1])
    expected = exp.copy()
    expected[bad] ^= 0x10
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    monkeypatch.setenv("TFS_CRC_VARIANT", "52")
    staged = crc.Context(0, measure=True)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    pin = crc.PinnedBuffer(gpu_ctx, size)
    try:
        pin.array[:] = data
        for rep in range(2):
            c1, ok1, nb1, rc1 = gpu_ctx.verify(pin.array, offs, lens, expected)
            c2, ok2, nb2, rc2 = gpu_ctx.verify(data.copy(), offs, lens, expected)
            c3, ok3, nb3, rc3 = staged.verify(pin.array, offs, lens, expected)
            assert (c1 == exp).all() and (c2 == exp).all() and (c3 == exp).all(), rep
            assert (ok1 == ok2).all() and (ok1 == ok3).all() and nb1 == nb2 == nb3 == len(bad), rep
            assert rc1 == rc2 == rc3 == -1010 and (ok1[bad] == 0).all(), rep
            c4, ok4, nb4, rc4 = gpu_ctx.verify(pin.array, offs, lens, exp)
            assert nb4 == 0 and rc4 == 0 and ok4.all() and (c4 == exp).all(), rep
        s1 = gpu_ctx.batch(pin.array, offs, lens, seeds)
        s2 = gpu_ctx.batch(data.copy(), offs, lens, seeds)
        assert (s1 == s2).all()
        for i in (0, 1, 4, 5, n // 2, n - 1):
            assert int(s1[i]) == ocrc(oracle, int(seeds[i]), data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
        # three submissions in flight over the same page-locked image, each wide
        parts = [np.arange(k, n, 3) for k in range(3)]
        hs = [gpu_ctx.submit_verify(pin.array, offs[p], lens[p], expected[p]) for p in parts]
        for p, h in zip(parts, hs):
            c, ok, nb, rc = gpu_ctx.wait(h)
            assert (c == exp[p]).all() and nb == int((ok == 0).sum()) == int(np.isin(p, bad).sum())
    finally:
        pin.free()
        staged.close()


@pytest.mark.parametrize("n", [65536, 65537])
def test_wide_pinned_batch_file_limit(gpu_ctx, oracle, n):
    """The in-place path for wide page-locked batches takes up to 65,536 files (the
    slot's page-locked verdict words); one file more goes the staged way.  Both
    sides of the limit: ragged small files with seeds (compute) and with planted
    mismatches (verify), every CRC against the oracle."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 300, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 5, n - 1).astype(np.uint64))
    size = int(offs[-1] + lens[-1]) + 64
    assert size > 8 << 20
    data = synth_bytes(7300 + n, size)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, seeds
    exp_s = np.zeros(n, np.uint32)
    oracle.oracle_crc_batch(d.ctypes.data, n, data.ctypes.data, exp_s.ctypes.data)
    d["aux"] = 0
    exp0 = np.zeros(n, np.uint32)
    oracle.oracle_crc_batch(d.ctypes.data, n, data.ctypes.data, exp0.ctypes.data)
    want = exp0.copy()
    bad = np.array([0, n // 2, n - 1])
    want[bad] ^= 0x40
    pin = crc.PinnedBuffer(gpu_ctx, size)
    try:
        pin.array[:] = data
        assert (gpu_ctx.batch(pin.array, offs, lens, seeds) == exp_s).all()
        c, ok, nb, rc = gpu_ctx.verify(pin.array, offs, lens, want)
        assert (c == exp0).all() and nb == 3 and rc == -1010 and not ok[bad].any() and ok.sum() == n - 3
    finally:
        pin.free()


def test_wide_pinned_batches_from_several_threads(gpu_ctx, oracle):
    """Four threads verify and compute over their own wide page-locked images (16 MiB,
    300 files each: the in-place throughput launch) on one context at once, 6 calls
    each, a mismatch planted per image: every result equals the oracle's."""
    import threading
    import tfs_amd.crc as crc
    rng = np.random.default_rng(9191)
    n = 300
    jobs = []
    for t in range(4):
        lens = rng.integers(20000, 90000, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)
        size = int(offs[-1] + lens[-1]) + 64
        data = synth_bytes(9200 + t, size)
        exp = np.array([ocrc(oracle, 0, data[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)],
                       np.uint32)
        want = exp.copy()
        want[t * 7] ^= 1
        pin = crc.PinnedBuffer(gpu_ctx, size)
        pin.array[:] = data
        jobs.append((pin, offs, lens, exp, want))
    errors = []

    def work(t):
        pin, offs, lens, exp, want = jobs[t]
        try:
            for it in range(6):
                c, ok, nb, rc = gpu_ctx.verify(pin.array, offs, lens, want)
                if not ((c == exp).all() and nb == 1 and rc == -1010 and not ok[t * 7]):
                    errors.append((t, it, "verify"))
                s = gpu_ctx.batch(pin.array, offs, lens, np.zeros(len(offs), np.uint32))
                if not (s == exp).all():
                    errors.append((t, it, "batch"))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))
    try:
        ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errors, errors
    finally:
        for j in jobs:
            j[0].free()


def test_small_pinned_batches_read_in_place(gpu_ctx, oracle):
    """tfs_crc32_verify / tfs_crc32_batch / submit+wait on a page-locked buffer whose
    span is <= 8 MiB run as one zero-copy launch (payloads, descriptors and verdicts in
    host memory, n_bad counted from the verdicts): same results as the staged pageable
    path and the oracle, ragged and empty files, several slots in flight."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(77)
    n = 300
    lens = rng.integers(0, 40000, n).astype(np.uint32)
    lens[:5] = [0, 1, 3, 4, 65536]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 7, n - 1).astype(np.uint64))
    size = int(offs[-1] + lens[-1]) + 16
    assert size <= 8 << 20
    data = rng.integers(0, 256, size, dtype=np.uint8)
    exp = np.array([ocrc(oracle, 0, data[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)], np.uint32)
    bad = np.array([7, 100, 299])
    expected = exp.copy()
    expected[bad] ^= 1
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    pin = crc.PinnedBuffer(gpu_ctx, size)
    try:
        pin.array[:] = data
        c1, ok1, nb1, rc1 = gpu_ctx.verify(pin.array, offs, lens, expected)
        c2, ok2, nb2, rc2 = gpu_ctx.verify(data.copy(), offs, lens, expected)
        assert (c1 == exp).all() and (c2 == exp).all()
        assert (ok1 == ok2).all() and nb1 == nb2 == len(bad) and rc1 == rc2 == -1010
        assert (ok1[bad] == 0).all() and ok1.sum() == n - len(bad)
        c3, ok3, nb3, rc3 = gpu_ctx.verify(pin.array, offs, lens, exp)
        assert nb3 == 0 and rc3 == 0 and ok3.all()
        s1 = gpu_ctx.batch(pin.array, offs, lens, seeds)
        s2 = gpu_ctx.batch(data.copy(), offs, lens, seeds)
        assert (s1 == s2).all()
        for i in (0, 1, 4, 150):
            assert int(s1[i]) == ocrc(oracle, int(seeds[i]), data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
        hs = [gpu_ctx.submit_verify(pin.array, offs[k::3], lens[k::3], expected[k::3]) for k in range(3)]
        for k, h in enumerate(hs):
            c, ok, nb, rc = gpu_ctx.wait(h)
            assert (c == exp[k::3]).all() and nb == int((ok == 0).sum()) == int(np.isin(np.arange(n)[k::3], bad).sum())
    finally:
        pin.free()


def test_pinned_registry_interior_bases_and_recycled_buffers(gpu_ctx, oracle):
    """Page-locked buffers the library allocated are found through its own registry
    (no HIP runtime query): a base in the middle of one is read in place at the right
    device address, and buffers freed and allocated again (maybe at the same address,
    with another size) are looked up afresh; pageable copies of the same bytes agree."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(5150)
    for rnd, size in enumerate((1 << 20, 3 << 19, 1 << 20, 5000)):
        pin = crc.PinnedBuffer(gpu_ctx, size)
        try:
            data = rng.integers(0, 256, size, dtype=np.uint8)
            pin.array[:] = data
            for skew in (0, 13, 4096 + 3):
                view = pin.array[skew:]
                n = 40
                lens = rng.integers(0, max(2, (size - skew) // n), n).astype(np.uint32)
                offs = np.zeros(n, np.uint64)
                offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
                assert int(offs[-1] + lens[-1]) <= view.size
                exp = np.array([ocrc(oracle, 0, view[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)],
                               np.uint32)
                c, ok, nb, rc = gpu_ctx.verify(view, offs, lens, exp)
                assert (c == exp).all() and ok.all() and nb == 0 and rc == 0, (rnd, skew)
                c2 = gpu_ctx.batch(view.copy(), offs, lens, np.zeros(n, np.uint32))
                assert (c2 == exp).all()
        finally:
            pin.free()


def test_device_resident_max_len_and_64bit_offsets(gpu_ctx, oracle):
    """Maximum sizes: one file of INT32_MAX bytes (Func::crc's `len` is int32, func.h:90)
    with a non-zero seed, a file straddling the 4 GiB offset boundary and one past 5 GiB
    (descriptor offsets are u64), computed and verified on the device; each checked
    against the oracle over the device's own bytes."""
    import ctypes
    import tfs_amd.crc as crc
    G = 1 << 30
    files = [(36, (1 << 31) - 1, 0x4E534654), (4 * G - 5, 100 * 1024 + 3, 0), (5 * G + 3, (1 << 20) + 7, 7)]
    nbytes = (5 * G + 3 + (1 << 20) + 7 + 4095) // 4096 * 4096
    img = crc.DeviceBuffer(gpu_ctx, nbytes)
    try:
        gpu_ctx.synth_fill_device(img, nbytes, 99, 0)
        d = np.zeros(len(files), crc.DESC_DTYPE)
        d["offset"] = [f[0] for f in files]
        d["len"] = [f[1] for f in files]
        d["aux"] = [f[2] for f in files]
        dd = crc.DeviceBuffer(gpu_ctx, d.nbytes).upload(d)
        out = crc.DeviceBuffer(gpu_ctx, 4 * len(files))
        gpu_ctx.batch_device(dd, len(files), img, out)
        gpu_ctx.sync()
        got = out.download(np.uint32)
        for i, (o, ln, seed) in enumerate(files):
            host = img.download(np.uint8, ln, o)
            want = oracle.oracle_crc(seed, ctypes.cast(host.ctypes.data, ctypes.c_char_p), ln)
            del host
            assert int(got[i]) == want, (i, hex(int(got[i])), hex(want))
        # verify-on-read starts from seed 0 (sync_backup.cpp:383): expected = crc(0, payload)
        z = d.copy()
        z["aux"] = 0
        zd = crc.DeviceBuffer(gpu_ctx, z.nbytes).upload(z)
        gpu_ctx.batch_device(zd, len(files), img, out)
        gpu_ctx.sync()
        v = d.copy()
        v["aux"] = out.download(np.uint32)
        assert int(v["aux"][1]) == int(got[1])                  # seed 0 there already
        v["aux"][0] ^= 0x80000000
        vd = crc.DeviceBuffer(gpu_ctx, v.nbytes).upload(v)
        okd = crc.DeviceBuffer(gpu_ctx, len(files))
        nb = crc.DeviceBuffer(gpu_ctx, 4)
        nb.zero()
        gpu_ctx.verify_device(vd, len(files), img, None, okd, nb)
        gpu_ctx.sync()
        assert int(nb.download(np.uint32)[0]) == 1 and okd.download().tolist() == [0, 1, 1]
    finally:
        img.free()


@pytest.mark.parametrize("variant", [0, 50])
def test_dynamic_tickets_verify_counts_each_file_once(oracle, variant, monkeypatch):
    """Verify over 1 M device-resident files on the dynamic (chunked) path with
    1,000 wrong expectations: n_bad is exactly 1,000 and the verdicts are 0 at
    exactly those files -- a file taken twice (or never) would show here."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(variant))
    ctx = crc.Context(0)
    try:
        rng = np.random.default_rng(5050 + variant)
        n = (1 << 20) + 333
        lens = rng.integers(0, 200, n)
        offs = np.cumsum(rng.integers(0, 8, n) + np.concatenate([[0], lens[:-1]])).astype(np.uint64)
        total = int(offs[-1] + lens[-1] + 64)
        buf = synth_bytes(6060 + variant, total)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"], d["len"] = offs, lens
        exp = np.zeros(n, np.uint32)
        oracle.oracle_crc_batch(d.ctypes.data, n, buf.ctypes.data, exp.ctypes.data)
        bad = rng.choice(n, 1000, replace=False)
        d["aux"] = exp
        d["aux"][bad] ^= 0x80000000
        img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096).upload(buf)
        dd = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
        okd = crc.DeviceBuffer(ctx, n)
        nb = crc.DeviceBuffer(ctx, 4)
        outc = crc.DeviceBuffer(ctx, 4 * n)
        okd.zero()
        nb.zero()
        ctx.verify_device(dd, n, img, outc, okd, nb)
        ctx.sync()
        assert int(nb.download(np.uint32)[0]) == 1000
        ok = okd.download(np.uint8, n)
        assert np.array_equal(np.sort(np.nonzero(ok == 0)[0]), np.sort(bad)) and (ok <= 1).all()
        assert np.array_equal(outc.download(np.uint32, n), exp)
    finally:
        ctx.close()


def test_wide_pinned_calls_from_threads_overlap_and_agree(gpu_ctx, oracle):
    """Round 6: each synchronous slot launches wide in-place batches on its own
    stream, so calls from several threads run side by side (the configs[2]
    receive-buffer leg: 3 caller threads).  Four threads x six calls each over
    three distinct page-locked images with split files, compute with seeds and
    verify with mismatches interleaved: every result equals the oracle's, and the
    context's later single-threaded calls still agree."""
    import threading
    import tfs_amd.crc as crc
    rng = np.random.default_rng(6006)
    imgs = []
    pins = []
    try:
        for k in range(3):
            n = 400 + 50 * k
            lens = rng.integers(1, 70000, n).astype(np.uint32)
            lens[3] = 400 * 1024 + k          # split files
            lens[n // 2] = (1 << 20) - 7
            offs = np.zeros(n, np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 97, n - 1).astype(np.uint64))
            size = int(offs[-1] + lens[-1]) + 64
            pin = crc.PinnedBuffer(gpu_ctx, size)
            pins.append(pin)
            pin.array[:] = rng.integers(0, 256, size, dtype=np.uint8)
            seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            d = np.zeros(n, crc.DESC_DTYPE)
            d["offset"], d["len"], d["aux"] = offs, lens, seeds
            exp_s = np.zeros(n, np.uint32)
            oracle.oracle_crc_batch(d.ctypes.data, n, pin.array.ctypes.data, exp_s.ctypes.data)
            d["aux"] = 0
            exp0 = np.zeros(n, np.uint32)
            oracle.oracle_crc_batch(d.ctypes.data, n, pin.array.ctypes.data, exp0.ctypes.data)
            imgs.append((pin, offs, lens, seeds, exp_s, exp0))
        errors = []

        def worker(t):
            try:
                for it in range(6):
                    pin, offs, lens, seeds, exp_s, exp0 = imgs[(t + it) % 3]
                    if (t + it) % 2:
                        got = gpu_ctx.batch(pin.array, offs, lens, seeds)
                        if not (got == exp_s).all():
                            errors.append(("batch", t, it, int((got != exp_s).sum())))
                    else:
                        want = exp0.copy()
                        want[it::97] ^= 1
                        c, ok, nb, rc = gpu_ctx.verify(pin.array, offs, lens, want)
                        nbad = len(range(it, len(want), 97))
                        if not ((c == exp0).all() and nb == nbad and int((ok == 0).sum()) == nbad):
                            errors.append(("verify", t, it, nb))
            except Exception as e:  # reported below
                errors.append(("exc", t, repr(e)))

        ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors[:5]
        pin, offs, lens, seeds, exp_s, exp0 = imgs[0]
        assert (gpu_ctx.batch(pin.array, offs, lens, seeds) == exp_s).all()
    finally:
        for p in pins:
            p.free()


def test_block_verify_in_place_from_threads(gpu_ctx, oracle):
    """Round 6: tfs_block_verify of a page-locked image runs on a synchronous
    slot's own stream with its wait outside the context lock, so verifies from
    several threads (the mirror, repair and checker call sites) run side by side.
    Four threads x five calls over three page-locked images with rejected records
    (payload CRC, FileInfo id, FileInfo size, too short, past the image): every
    call's statuses and CRCs equal the single-threaded call's, which the oracle
    pins record by record."""
    import ctypes
    import threading
    import tfs_amd.crc as crc
    rng = np.random.default_rng(6116)
    cases = []
    pins = []
    try:
        for k in range(3):
            sizes = [int(x) for x in rng.choice([1, 100, 4096, 65536, 70001, 200000], 40)]
            img, metas = _block_image(oracle, sizes, seed=6200 + k)
            img[int(metas[3]["offset"]) + 36 + 5] ^= 0x20        # payload CRC
            metas[7]["file_id"] += 1                               # FileInfo id
            img[int(metas[9]["offset"]) + 12] ^= 0x01             # FileInfo size
            metas[11]["size"] = 36                                 # too short
            metas[13]["offset"] = img.size - 10                    # past the image
            pin = crc.PinnedBuffer(gpu_ctx, img.size)
            pins.append(pin)
            pin.array[:] = img
            c, st, nb, rc = gpu_ctx.block_verify(pin.array, metas)
            for i in range(len(sizes)):
                oc = ctypes.c_uint32()
                code = oracle.oracle_verify_file(pin.ptr, img.size, int(metas[i]["offset"]), int(metas[i]["size"]),
                                                 ctypes.byref(oc))
                if i in (7, 11):  # the id and short-record checks come before the oracle's helper's
                    assert st[i] == (-8016 if i == 7 else -8034), (k, i, st[i])
                    continue
                assert code == st[i], (k, i, code, st[i])
                if code in (0, -1010):
                    assert int(c[i]) == oc.value, (k, i)
            cases.append((pin, metas, c.copy(), st.copy(), nb))
        errors = []

        def worker(t):
            try:
                for it in range(5):
                    pin, metas, c0, st0, nb0 = cases[(t + it) % 3]
                    c, st, nb, rc = gpu_ctx.block_verify(pin.array, metas)
                    if not ((st == st0).all() and nb == nb0 and (c[st0 == 0] == c0[st0 == 0]).all()):
                        errors.append((t, it))
            except Exception as e:
                errors.append(("exc", t, repr(e)))

        ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors[:5]
    finally:
        for p in pins:
            p.free()
