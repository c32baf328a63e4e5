"""The compaction data pass under every kernel form: the product
pipelined kernel (dynamic tickets, next-record prefetch, DPP lane shifts, the
hybrid static/ticketed record order) and the round-5 occupancy forms of the
measurement build (TFS_CRC_VARIANT 94-99: two workgroups per CU over 74 KiB of
LDS tables, and its one-workgroup control 97).  Each must produce the oracle's
real_compact bytes and statuses exactly, for every destination shift class, tiny
and large records, rejected records (size, range, id, CRC), device-resident
single-block and many-block forms, and zero-copy host images."""
import numpy as np
import pytest

from conftest import ocrc
from test_gpu_parity import _block_image, _oracle_compact


def ocrc_payload(oracle, img, meta):
    o = int(meta["offset"]) + 36
    return ocrc(oracle, 0, img[o:o + int(meta["size"]) - 36].tobytes())

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 94, 95, 96, 97, 98, 99, 120, 121])
def vctx(request, monkeypatch):
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(request.param))
    ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    yield ctx
    ctx.close()


def _shift_class_block(oracle, seed, n=200):
    rng = np.random.default_rng(seed)
    sizes, flags = [], []
    for k in range(n):
        sizes.append(int(rng.choice([1, 3, 17, 31, 32, 33, 100, 1023, 1024, 1025, 2049, 5000, 65536, 70001,
                                     200000])))
        flags.append(1 if k % 3 == 1 else 0)
        if flags[-1]:
            sizes[-1] = 16 + (k % 16 - 36) % 16 + 16 * int(rng.integers(0, 4))
    img, metas = _block_image(oracle, sizes, seed=seed)
    return img, metas, np.array(flags, np.int32)


def test_host_compaction_all_shift_classes(vctx, oracle):
    img, metas, fl = _shift_class_block(oracle, 301)
    assert fl[9] == 0
    img[int(metas[9]["offset"]) + 36 + 3] ^= 0x80     # a live record with a bad payload
    dest, dmetas, ok, rc = vctx.block_compact(img, metas, fl)
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    assert dest.size == odest.size and (dest == odest).all()
    assert (ok == ook).all() and rc == -1010


def test_device_compaction_statuses(vctx, oracle):
    """tfs_block_compact_device with rejected records mixed in: too short, past the
    image, wrong FileInfo id, wrong FileInfo size, bad CRC -- statuses in the
    reference's order (id, size, crc), good records repacked byte-exact."""
    import tfs_amd.crc as crc
    img, metas, fl = _shift_class_block(oracle, 302, 120)
    live = np.nonzero(fl == 0)[0]
    lm = np.ascontiguousarray(metas[live])
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    ld = np.concatenate([[0], np.cumsum(lm["size"].astype(np.int64))[:-1]]).astype(np.int64)
    bad = {}
    lm[3]["size"] = 35                       # shorter than its FileInfo
    bad[3] = -8034
    lm[5]["offset"] = img.size - 8           # runs past the image
    bad[5] = -1016
    lm[7]["file_id"] = 123456789             # FileInfo id != index
    bad[7] = -8016
    img2 = img.copy()
    img2[int(lm[9]["offset"]) + 12] ^= 1     # FileInfo.size_ != index size
    bad[9] = -8038
    img2[int(lm[11]["offset"]) + 36] ^= 1    # payload corrupted
    bad[11] = -1010
    n = len(lm)
    d_src = crc.DeviceBuffer(vctx, img2.size + 64).upload(img2)
    d_m = crc.DeviceBuffer(vctx, lm.nbytes).upload(lm)
    d_f = crc.DeviceBuffer(vctx, 4 * n).upload(np.zeros(n, np.int32))
    d_o = crc.DeviceBuffer(vctx, 8 * n).upload(ld)
    d_dst = crc.DeviceBuffer(vctx, odest.size + 64)
    d_dst.zero()
    d_st = crc.DeviceBuffer(vctx, 4 * n)
    d_bad = crc.DeviceBuffer(vctx, 4)
    d_bad.zero()
    vctx.block_compact_device(d_src, img2.size, d_m, d_f, d_o, n, d_dst, None, d_st, d_bad)
    vctx.sync()
    st = d_st.download(np.int32, n)
    out = d_dst.download(np.uint8, odest.size)
    for k in range(n):
        assert st[k] == bad.get(k, 0), (k, st[k])
        if k in bad:
            continue
        o, sz = int(ld[k]), int(lm[k]["size"])
        assert (out[o:o + sz] == odest[o:o + sz]).all(), k
    assert int(d_bad.download(np.uint32, 1)[0]) == len(bad)


def test_jobs_device_many_blocks_shuffled(vctx, oracle):
    import tfs_amd.crc as crc
    rng = np.random.default_rng(303)
    blocks, jobs, expect = [], [], []
    src_base = dst_base = 0
    for b in range(6):
        img, metas, fl = _shift_class_block(oracle, 310 + b, 60)
        odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
        for i in np.nonzero((fl & 3) == 0)[0]:
            jobs.append((src_base + int(metas[i]["offset"]), dst_base + int(doff[i]), int(metas[i]["file_id"]),
                         int(metas[i]["size"]), 0, int(doff[i]), 0))
        blocks.append(img[:int(metas["size"].astype(np.int64).sum())])
        expect.append((dst_base, odest))
        src_base += blocks[-1].size
        dst_base += odest.size + (b * 5) % 16
    src = np.concatenate(blocks)
    j = np.array(jobs, dtype=crc.COMPACT_JOB_DTYPE)
    rng.shuffle(j)
    d_src = crc.DeviceBuffer(vctx, src.size + 64).upload(src)
    d_j = crc.DeviceBuffer(vctx, j.nbytes).upload(j)
    d_dst = crc.DeviceBuffer(vctx, dst_base + 64)
    d_dst.zero()
    d_st = crc.DeviceBuffer(vctx, 4 * len(j))
    d_bad = crc.DeviceBuffer(vctx, 4)
    d_bad.zero()
    for rep in range(3):   # repeated launches on one stream: tickets reset by each launch
        vctx.compact_jobs_device(d_src, src.size, d_j, len(j), d_dst, None, d_st, d_bad)
    vctx.sync()
    out = d_dst.download(np.uint8, dst_base)
    for base, od in expect:
        assert (out[base:base + od.size] == od).all()
    assert int(d_bad.download(np.uint32, 1)[0]) == 0 and (d_st.download(np.int32, len(j)) == 0).all()


def test_jobs_device_statuses_and_split_records(vctx, oracle):
    _jobs_statuses_case(vctx, oracle)


@pytest.mark.parametrize("seg", [8192, 16384, 32768, 0])
def test_product_segmented_compaction_toggle(gpu_ctx, oracle, seg):
    """The product library with tfs_crc32_set_compact_segment: every segment size
    and back to whole records on the same context, same results."""
    gpu_ctx.set_compact_segment(seg)
    try:
        _jobs_statuses_case(gpu_ctx, oracle)
        # every record flagged TFS_COMPACT_JOB_EDGE (the bit rides on a
        # split record's last segment): the same bytes, CRCs and statuses
        _jobs_statuses_case(gpu_ctx, oracle, edge=True)
    finally:
        gpu_ctx.set_compact_segment(1)  # the default again (whole records)
    with pytest.raises(Exception):
        gpu_ctx.set_compact_segment(12345)


def _jobs_statuses_case(vctx, oracle, edge=False):
    """tfs_compact_jobs_device over records of every size class (many longer than
    the 8 / 16 / 32 KiB segments of the segmented form, including exact
    multiples and one byte past them), with rejected records on both short and
    long records: FileInfo id, FileInfo size, payload CRC (in a later segment and
    in the head), too short, past the image.  Statuses in the reference's order,
    CRCs of every checked record equal to the oracle's, good records byte-exact."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(330)
    sizes = [int(x) for x in rng.choice([1, 33, 1024, 8191, 8192, 8193, 16384, 16385, 32768, 32769, 65536, 70001,
                                          200000, 300001], 160)]
    sizes[:6] = [8193, 16385, 32769, 98304, 98305, 262144]
    img, metas = _block_image(oracle, sizes, seed=331)
    n = len(sizes)
    fl = np.zeros(n, np.int32)
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    crcs = np.array([ocrc_payload(oracle, img, metas[k]) for k in range(n)], np.uint32)
    j = np.zeros(n, crc.COMPACT_JOB_DTYPE)
    j["src_offset"], j["dest_offset"] = metas["offset"], doff
    j["file_id"], j["size"], j["new_offset"] = metas["file_id"], metas["size"], doff
    if edge:
        j["reserved"] = 1   # TFS_COMPACT_JOB_EDGE: no byte past any record is read
    big = [k for k in range(n) if sizes[k] > 40000]
    bad = {}
    img2 = img.copy()
    j["file_id"][big[0]] += 7                                  # id mismatch on a long record
    bad[big[0]] = -8016
    img2[int(metas[big[1]]["offset"]) + 12] ^= 1               # FileInfo.size_ mismatch on a long record
    bad[big[1]] = -8038
    img2[int(metas[big[2]]["offset"]) + 36 + sizes[big[2]] - 5] ^= 0x10   # CRC: last segment
    bad[big[2]] = -1010
    img2[int(metas[big[3]]["offset"]) + 36 + 2] ^= 0x01        # CRC: head bytes
    bad[big[3]] = -1010
    j["size"][10] = 30                                         # shorter than a FileInfo
    bad[10] = -8034
    j["src_offset"][11] = img.size - 100                       # past the image
    bad[11] = -1016
    d_src = crc.DeviceBuffer(vctx, img2.size + 64).upload(img2)
    d_j = crc.DeviceBuffer(vctx, j.nbytes).upload(j)
    d_dst = crc.DeviceBuffer(vctx, odest.size + 64)
    d_dst.zero()
    d_st = crc.DeviceBuffer(vctx, 4 * n)
    d_c = crc.DeviceBuffer(vctx, 4 * n)
    d_bad = crc.DeviceBuffer(vctx, 4)
    for rep in range(2):  # twice on one stream: the plan and the slot are reused
        d_bad.zero()
        vctx.compact_jobs_device(d_src, img2.size, d_j, n, d_dst, d_c, d_st, d_bad)
        vctx.sync()
        st = d_st.download(np.int32, n)
        c = d_c.download(np.uint32, n)
        out = d_dst.download(np.uint8, odest.size)
        for k in range(n):
            assert st[k] == bad.get(k, 0), (rep, k, sizes[k], st[k])
            if k in (10, 11):
                continue
            if bad.get(k) == -1010:
                pl = img2[int(metas[k]["offset"]) + 36:int(metas[k]["offset"]) + 36 + sizes[k]]
                assert c[k] == ocrc(oracle, 0, pl.tobytes()), (rep, k)
            else:
                assert c[k] == crcs[k], (rep, k, sizes[k])
            if k in bad:
                continue
            o, sz = int(doff[k]), int(metas[k]["size"])
            assert (out[o:o + sz] == odest[o:o + sz]).all(), (rep, k, sizes[k])
        assert int(d_bad.download(np.uint32, 1)[0]) == len(bad)


def test_zero_copy_host_images(vctx, oracle):
    import tfs_amd.crc as crc
    img, metas = _block_image(oracle, [65536] * 40 + [4 * 777, 4 * 1001], seed=320)
    fl = np.zeros(len(metas), np.int32)
    fl[::2] = 1
    src = crc.PinnedBuffer(vctx, img.size)
    cap = int(metas["size"].astype(np.int64).sum()) + 64
    dst = crc.PinnedBuffer(vctx, cap)
    try:
        src.array[:] = img
        dst.array[:] = 0
        jobs = (crc.BlockJob * 1)()
        ok = np.zeros(len(metas), np.uint8)
        j = jobs[0]
        j.src_image, j.src_len, j.metas, j.flags, j.n = src.ptr, img.size, metas.ctypes.data, fl.ctypes.data, len(metas)
        j.dest_image, j.dest_cap, j.crc_ok = dst.ptr, cap, ok.ctypes.data
        assert vctx.blocks_compact(jobs) == 0
        odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
        assert (dst.array[:odest.size] == odest).all() and (ok == ook).all()
    finally:
        src.free()
        dst.free()


@pytest.fixture(params=[0, 50])
def vfy_ctx(request, monkeypatch):
    """Verify-on-read forms: the pipelined record kernel (product: chunked tickets)
    and one record per ticket (TFS_CRC_VARIANT=50)."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(request.param))
    ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    yield ctx
    ctx.close()


def _statuses_case(oracle):
    img, metas, fl = _shift_class_block(oracle, 330, 160)
    m = np.ascontiguousarray(metas.copy())
    img = img.copy()
    m[2]["size"] = 20                                 # too short      -> -8034
    m[4]["offset"] = img.size - 10                    # past the image -> -1016
    m[6]["file_id"] = 999                             # id mismatch    -> -8016
    img[int(m[8]["offset"]) + 12] ^= 2                # size mismatch  -> -8038
    img[int(m[10]["offset"]) + 36 + int(m[10]["size"]) // 2 - 18] ^= 1   # bad payload -> -1010
    want = {2: -8034, 4: -1016, 6: -8016, 8: -8038, 10: -1010}
    return img, m, want


def test_block_verify_forms_statuses(vfy_ctx, oracle):
    import tfs_amd.crc as crc
    img, m, want = _statuses_case(oracle)
    for k in range(len(m)):
        if k in want:
            continue
        o, sz = int(m[k]["offset"]), int(m[k]["size"])
        assert oracle.oracle_verify_file(img.ctypes.data, img.size, o, sz, None) == 0
    # host form
    c, st, nbad, rc = vfy_ctx.block_verify(img, m)
    assert rc == -1010 and nbad == len(want)
    assert {k: int(st[k]) for k in range(len(m)) if st[k] != 0} == want
    for k in range(len(m)):
        if st[k] == 0:
            o, sz = int(m[k]["offset"]), int(m[k]["size"])
            oc = __import__("ctypes").c_uint32()
            oracle.oracle_verify_file(img.ctypes.data, img.size, o, sz, __import__("ctypes").byref(oc))
            assert int(c[k]) == oc.value
    # device form
    n = len(m)
    d_img = crc.DeviceBuffer(vfy_ctx, img.size + 64).upload(img)
    d_m = crc.DeviceBuffer(vfy_ctx, m.nbytes).upload(m)
    d_c = crc.DeviceBuffer(vfy_ctx, 4 * n)
    d_s = crc.DeviceBuffer(vfy_ctx, 4 * n)
    d_b = crc.DeviceBuffer(vfy_ctx, 4)
    d_b.zero()
    vfy_ctx.block_verify_device(d_img, img.size, d_m, n, d_c, d_s, d_b)
    vfy_ctx.sync()
    assert (d_s.download(np.int32, n) == st).all() and (d_c.download(np.uint32, n)[st == 0] == c[st == 0]).all()
    assert int(d_b.download(np.uint32, 1)[0]) == len(want)


def test_blocks_verify_device_many_blocks(gpu_ctx, oracle):
    """tfs_blocks_verify_device: records of several blocks (64-bit offsets, any order)
    in one launch, statuses as the single-block form."""
    import tfs_amd.crc as crc
    imgs, jobs, want = [], [], []
    base = 0
    for b in range(4):
        img, m, w = _statuses_case(oracle) if b == 2 else (*_shift_class_block(oracle, 340 + b, 80)[:2], {})
        for k in range(len(m)):
            jobs.append((base + max(int(m[k]["offset"]), 0) if int(m[k]["offset"]) >= 0 else 0, 0,
                         int(m[k]["file_id"]), int(m[k]["size"]), 0, 0, 0))
            want.append(w.get(k, 0))
        imgs.append(img)
        base += img.size
    src = np.concatenate(imgs)
    # the "past the image" record of block 2 must be past the whole buffer here
    j = np.array(jobs, dtype=crc.COMPACT_JOB_DTYPE)
    idx = [i for i, x in enumerate(want) if x == -1016]
    j["src_offset"][idx] = src.size - 10
    order = np.random.default_rng(5).permutation(len(j))
    j, want = j[order], np.array(want, np.int32)[order]
    n = len(j)
    d_src = crc.DeviceBuffer(gpu_ctx, src.size + 64).upload(src)
    d_j = crc.DeviceBuffer(gpu_ctx, j.nbytes).upload(j)
    d_s = crc.DeviceBuffer(gpu_ctx, 4 * n)
    d_b = crc.DeviceBuffer(gpu_ctx, 4)
    d_b.zero()
    gpu_ctx.blocks_verify_device(d_src, src.size, d_j, n, None, d_s, d_b)
    gpu_ctx.sync()
    assert (d_s.download(np.int32, n) == want).all()
    assert int(d_b.download(np.uint32, 1)[0]) == int((want != 0).sum())


@pytest.fixture(scope="module")
def many_records(oracle):
    """420 k short records (1..300-byte payloads) in one image, every third deleted:
    enough records per wave for the dynamic-ticket path with chunks of up to 4."""
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes
    rng = np.random.default_rng(350)
    n = 420_000
    sizes = rng.integers(1, 301, n)
    recs = sizes + 36
    offs = np.concatenate([[0], np.cumsum(recs)[:-1]]).astype(np.int64)
    img = synth_bytes(351, int(recs.sum()) + 64).copy()
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"] = offs + 36, sizes
    c = np.zeros(n, np.uint32)
    oracle.oracle_crc_batch(d.ctypes.data, n, img.ctypes.data, c.ctypes.data)
    fi = np.zeros(n, crc.FILEINFO_DTYPE)
    fi["id_"] = 1000 + np.arange(n)
    fi["offset_"] = offs
    fi["size_"] = fi["usize_"] = recs
    fi["crc_"] = c
    img[offs[:, None] + np.arange(36)[None, :]] = fi.view(np.uint8).reshape(n, 36)
    metas = np.zeros(n, crc.META_DTYPE)
    metas["file_id"], metas["offset"], metas["size"] = 1000 + np.arange(n), offs, recs
    fl = np.zeros(n, np.int32)
    fl[1::3] = 1
    return img, metas, fl, c


@pytest.fixture(params=[0, 50, 94, 99])
def chunk_ctx(request, monkeypatch):
    """The product record kernel, one record per ticket on verify (50) and two
    occupancy forms of the compaction (94, 99)."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", str(request.param))
    ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    yield ctx
    ctx.close()


def test_dynamic_tickets_many_records(chunk_ctx, oracle, many_records):
    """Compaction (jobs form) and verify-on-read (jobs form) over 280 k / 420 k
    records in one launch each: byte-exact against the oracle's real_compact and
    its CRCs, every status 0."""
    import tfs_amd.crc as crc
    img, metas, fl, c = many_records
    odest, doff, ook = _oracle_compact(oracle, img, metas, fl)
    live = np.nonzero(fl == 0)[0]
    j = np.zeros(live.size, crc.COMPACT_JOB_DTYPE)
    j["src_offset"], j["dest_offset"] = metas["offset"][live], doff[live]
    j["file_id"], j["size"], j["new_offset"] = metas["file_id"][live], metas["size"][live], doff[live]
    d_src = crc.DeviceBuffer(chunk_ctx, img.size + 64).upload(img)
    d_j = crc.DeviceBuffer(chunk_ctx, j.nbytes).upload(j)
    d_dst = crc.DeviceBuffer(chunk_ctx, odest.size + 64)
    d_dst.zero()
    d_st = crc.DeviceBuffer(chunk_ctx, 4 * len(metas))
    d_c = crc.DeviceBuffer(chunk_ctx, 4 * len(metas))
    d_bad = crc.DeviceBuffer(chunk_ctx, 4)
    d_bad.zero()
    chunk_ctx.compact_jobs_device(d_src, img.size, d_j, live.size, d_dst, None, d_st, d_bad)
    chunk_ctx.sync()
    assert int(d_bad.download(np.uint32, 1)[0]) == 0 and (d_st.download(np.int32, live.size) == 0).all()
    assert (d_dst.download(np.uint8, odest.size) == odest).all()
    n = len(metas)
    jv = np.zeros(n, crc.COMPACT_JOB_DTYPE)
    jv["src_offset"], jv["file_id"], jv["size"] = metas["offset"], metas["file_id"], metas["size"]
    d_jv = crc.DeviceBuffer(chunk_ctx, jv.nbytes).upload(jv)
    chunk_ctx.blocks_verify_device(d_src, img.size, d_jv, n, d_c, d_st, d_bad)
    chunk_ctx.sync()
    assert int(d_bad.download(np.uint32, 1)[0]) == 0 and (d_st.download(np.int32, n) == 0).all()
    assert (d_c.download(np.uint32, n) == c).all()


@pytest.mark.parametrize("variant", [0, 94, 95, 96, 97, 98, 99])
def test_hybrid_static_then_ticket_order_long_launch(oracle, variant, monkeypatch):
    """The product's record order (FileCursor HS): a launch of >= 16 records per
    wave hands the first n - (n >> HS) records out statically and the rest by
    tickets -- both phases must cover every record exactly once, also over the
    10-, 12- and 16-wave workgroups of the occupancy forms (94-99).  100 k records,
    most of 0.5-2 KiB payload and one in twenty of 33-100 KiB, every fourth
    deleted, byte-exact against the oracle's real_compact with CRCs and statuses."""
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes
    from test_headline_parity import _oracle_mt
    monkeypatch.setenv("TFS_CRC_VARIANT", str(variant))
    ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    rng = np.random.default_rng(variant)
    n = 100_000
    sizes = rng.integers(512, 2049, n)
    big = rng.random(n) < 0.05
    sizes[big] = rng.integers(33 << 10, 100 << 10, int(big.sum()))
    recs = sizes + 36
    offs = np.concatenate([[0], np.cumsum(recs)[:-1]]).astype(np.int64)
    img = synth_bytes(3000 + variant, int(recs.sum()) + 256)
    c = _oracle_mt(oracle, img, offs + 36, sizes)
    fi = np.zeros(n, crc.FILEINFO_DTYPE)
    fi["id_"] = 9000 + np.arange(n)
    fi["offset_"], fi["size_"], fi["usize_"], fi["crc_"] = offs, recs, recs, c
    img[offs[:, None] + np.arange(36)[None, :]] = fi.view(np.uint8).reshape(n, 36)
    metas = np.zeros(n, crc.META_DTYPE)
    metas["file_id"], metas["offset"], metas["size"] = 9000 + np.arange(n), offs, recs
    fl = np.zeros(n, np.int32)
    fl[1::4] = 1
    odest, doff, _ = _oracle_compact(oracle, img, metas, fl)
    live = np.nonzero(fl == 0)[0]
    assert live.size >= 16 * 4096
    j = np.zeros(live.size, crc.COMPACT_JOB_DTYPE)
    j["src_offset"], j["dest_offset"] = metas["offset"][live], doff[live]
    j["file_id"], j["size"], j["new_offset"] = metas["file_id"][live], metas["size"][live], doff[live]
    bufs = [crc.DeviceBuffer(ctx, img.size).upload(img), crc.DeviceBuffer(ctx, j.nbytes).upload(j),
            crc.DeviceBuffer(ctx, odest.size + 64), crc.DeviceBuffer(ctx, 4 * live.size),
            crc.DeviceBuffer(ctx, 4 * live.size), crc.DeviceBuffer(ctx, 4)]
    d_src, d_j, d_dst, d_c, d_st, d_nb = bufs
    try:
        d_dst.zero()
        d_nb.zero()
        d_st.zero()
        ctx.compact_jobs_device(d_src, img.size, d_j, live.size, d_dst, d_c, d_st, d_nb)
        ctx.sync()
        assert int(d_nb.download(np.uint32)[0]) == 0 and (d_st.download(np.int32, live.size) == 0).all()
        assert (d_c.download(np.uint32, live.size) == c[live]).all()
        assert (d_dst.download(np.uint8, odest.size) == odest).all()
    finally:
        for b in bufs:
            b.free()
        ctx.close()
