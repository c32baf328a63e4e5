"""On-disk block formats: tfs_amd/ds/block_store.{h,cpp}.

Physical block files with BlockPrefix chains (physical_block.cpp:30-60,172-189),
main/extension stitching (data_handle.cpp:103-141), the hash index
(index_handle.cpp:844-878,1015-1060) and real flags (logic_block.cpp:996-1009,
1250-1273).  Parity note: there is no block file written by the reference in
/root/reference (the dataserver cannot be built here: tbsys/tbnet are absent),
so the format is pinned by the reference's struct definitions and write path,
restated in the writer; the reader is checked against it and against hand-made
variants (prefix file, hash collisions, broken chains).  Verify-from-disk is
checked against the oracle on the GPU.
"""
import os
import struct

import numpy as np
import pytest

from tests.conftest import ocrc
from tfs_amd.synth import synth_bytes

MiB = 1 << 20


@pytest.fixture(scope="module")
def ds():
    from tfs_amd import dataserver
    dataserver.lib()
    return dataserver


def make_block(ds, oracle, block_id, sizes, seed=1, flags=None):
    b = ds.LogicBlock(block_id)
    for i, ln in enumerate(sizes):
        payload = synth_bytes(seed * 1000 + i, ln).tobytes()
        assert b.append(i + 1, payload, ocrc(oracle, 0, payload)) == 0
    for fid, fl in (flags or {}).items():
        assert b.set_flag(fid, fl) == 0
    return b


def check_loaded(ds, block, lb, flags=None):
    assert lb.rc == 0
    assert np.array_equal(lb.data(), block.raw())
    m, _ = block.metas()
    assert np.array_equal(lb.metas, m)
    exp = np.zeros(len(m), np.int32)
    for fid, fl in (flags or {}).items():
        exp[np.nonzero(m["file_id"] == fid)[0][0]] = fl
    assert np.array_equal(lb.flags, exp)


def test_roundtrip_chain_and_index(ds, oracle, tmp_path):
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(0, 60000, 80)]
    flags = {3: 1, 10: 1, 11: 4, 40: 5}
    blk = make_block(ds, oracle, 77, sizes, flags=flags)
    mount = str(tmp_path)
    ext = ds.write_block_files(blk, mount, main_id=5, first_ext_id=100, bucket_size=13, main_size=1 * MiB,
                               ext_size=256 * 1024)
    total = int(blk.raw().size)
    assert len(ext) == -(-(total - (MiB - 512)) // (256 * 1024 - 512))
    lb = ds.LoadedBlock(None, mount, 5, main_size=1 * MiB, ext_size=256 * 1024)
    check_loaded(ds, blk, lb, flags)
    assert lb.chain == [5] + ext and lb.logic_block_id == 77
    h = lb.header[0]
    assert h["bucket_size"] == 13 and h["data_file_offset"] == total and h["file_count"] == len(sizes)
    assert h["index_file_size"] == 48 + 4 * 13 + 20 * len(sizes)
    assert h["del_file_count"] == sum(1 for f in flags.values() if f & 1)
    # the files are TFS-shaped: <mount>/<main>, <mount>/extend/<id>, <mount>/index/<main>
    assert os.path.getsize(os.path.join(mount, "5")) == MiB
    assert os.path.getsize(os.path.join(mount, "extend", str(ext[0]))) == 256 * 1024
    raw = open(os.path.join(mount, "5"), "rb").read(24)
    assert struct.unpack("<IIIIQ", raw) == (77, 0, ext[0], 0, 0)


def test_index_entries_carry_unlink_flags(ds, oracle, tmp_path):
    blk = make_block(ds, oracle, 9, [100] * 6, flags={2: 1, 5: 2})
    mount = str(tmp_path)
    ds.write_block_files(blk, mount, 1, 50, bucket_size=4)
    idx = open(os.path.join(mount, "index", "1"), "rb").read()
    sizes = {}
    for pos in range(48 + 16, len(idx), 20):
        fid, off, sz, nxt = struct.unpack_from("<Qiii", idx, pos)
        sizes[fid] = sz
    assert sizes[2] == (136 | 0x08000000 | (1 << 28)) and sizes[5] == (136 | 0x08000000 | (2 << 28))
    assert sizes[1] == 136  # untouched entries keep the plain size
    # FileInfo.flag_ on disk stays 0 (unlink_file writes the flag to the index only)
    data = open(os.path.join(mount, "1"), "rb").read()
    assert struct.unpack_from("<i", data, 512 + 136 + 28)[0] == 0


def test_block_prefix_file_and_collisions(ds, oracle, tmp_path):
    blk = make_block(ds, oracle, 31, [5000] * 40, seed=2)
    mount = str(tmp_path)
    ext = ds.write_block_files(blk, mount, 3, 7, bucket_size=3, main_size=64 * 1024, ext_size=32 * 1024)
    # move every prefix into <mount>/block_prefix at (id-1)*24 and wipe the in-file copies
    pf = bytearray(24 * (max([3] + ext) + 1))
    for pid, path in [(3, os.path.join(mount, "3"))] + [(e, os.path.join(mount, "extend", str(e))) for e in ext]:
        with open(path, "r+b") as f:
            pf[(pid - 1) * 24:pid * 24] = f.read(24)
            f.seek(0)
            f.write(b"\0" * 24)
    open(os.path.join(mount, "block_prefix"), "wb").write(bytes(pf))
    lb = ds.LoadedBlock(None, mount, 3, main_size=64 * 1024, ext_size=32 * 1024)
    check_loaded(ds, blk, lb)
    assert lb.chain == [3] + ext


def test_broken_chain_and_index_rejected(ds, oracle, tmp_path):
    blk = make_block(ds, oracle, 8, [3000] * 30, seed=3)
    mount = str(tmp_path)
    ext = ds.write_block_files(blk, mount, 2, 20, bucket_size=5, main_size=32 * 1024, ext_size=16 * 1024)
    with open(os.path.join(mount, "extend", str(ext[1])), "r+b") as f:  # wrong back link
        f.seek(4)
        f.write(struct.pack("<I", 999))
    assert ds.LoadedBlock(None, mount, 2, main_size=32 * 1024, ext_size=16 * 1024).rc != 0
    blk2 = make_block(ds, oracle, 8, [3000] * 30, seed=3)
    m2 = str(tmp_path / "b")
    ds.write_block_files(blk2, m2, 2, 20, bucket_size=5, main_size=32 * 1024, ext_size=16 * 1024)
    with open(os.path.join(m2, "index", "2"), "r+b") as f:  # bucket pointing past the index
        f.seek(48)
        f.write(struct.pack("<i", 1 << 20))
    assert ds.LoadedBlock(None, m2, 2, main_size=32 * 1024, ext_size=16 * 1024).rc != 0


def baseline_block(ds, oracle):
    """1,024 x 64 KiB files in a 64 MiB main block; the 1,024th spills
    37,376 B into an extension block."""
    return make_block(ds, oracle, 4242, [65536] * 1024, seed=9)


def test_baseline_layout_spills_into_ext(ds, oracle, tmp_path):
    blk = baseline_block(ds, oracle)
    mount = str(tmp_path)
    ext = ds.write_block_files(blk, mount, 11, 500)
    assert len(ext) == 1
    assert blk.raw().size - (64 * MiB - 512) == 37376
    lb = ds.LoadedBlock(None, mount, 11)
    check_loaded(ds, blk, lb)


@pytest.mark.gpu
def test_gpu_verify_block_files(ds, oracle, gpu_ctx, tmp_path):
    blk = baseline_block(ds, oracle)
    blk.set_flag(100, 1)  # deleted: skipped
    mount = str(tmp_path)
    ext = ds.write_block_files(blk, mount, 11, 500)
    checker = ds.BlockCrcChecker(4)
    rc, st = ds.verify_block_files(gpu_ctx, mount, 11, checker)
    assert rc == 0 and len(st) == 1023 and (st == 0).all()
    # corrupt the payload of the last file where it lies in the extension block,
    # and one file in the main block
    with open(os.path.join(mount, "extend", str(ext[0])), "r+b") as f:
        f.seek(512 + 1000)
        b = f.read(1)
        f.seek(512 + 1000)
        f.write(bytes([b[0] ^ 0x20]))
    m, _ = blk.metas()
    off7 = int(m["offset"][7]) + 36 + 5
    with open(os.path.join(mount, "11"), "r+b") as f:
        f.seek(512 + off7)
        b = f.read(1)
        f.seek(512 + off7)
        f.write(bytes([b[0] ^ 0x01]))
    rc, st = ds.verify_block_files(gpu_ctx, mount, 11, checker)
    assert rc == 2
    assert st[7] == -1010 and st[-1] == -1010
    assert (np.delete(st, [7, len(st) - 1]) == 0).all()
    assert checker.errors(4242) == 2
    # oracle on the stitched image agrees file by file
    lb = ds.LoadedBlock(None, mount, 11)
    img = lb.data().tobytes()
    live = [i for i in range(len(lb.metas)) if lb.flags[i] == 0]
    for k, i in enumerate(live):
        o, sz = int(lb.metas["offset"][i]), int(lb.metas["size"][i])
        stored = struct.unpack_from("<I", img, o + 32)[0]
        exp = 0 if ocrc(oracle, 0, img[o + 36:o + sz]) == stored else -1010
        assert st[k] == exp


def _flip_on_disk(mount, chain, main_size, ext_size, logic_off, mask=0x40):
    """Flip bits of one byte at a logic data offset, in the physical block that holds it."""
    base = 0
    for k, pid in enumerate(chain):
        area = (main_size if k == 0 else ext_size) - 512
        if logic_off < base + area:
            path = os.path.join(mount, str(pid)) if k == 0 else os.path.join(mount, "extend", str(pid))
            with open(path, "r+b") as f:
                f.seek(512 + logic_off - base)
                b = f.read(1)
                f.seek(512 + logic_off - base)
                f.write(bytes([b[0] ^ mask]))
            return
        base += area
    raise AssertionError("offset past the chain")


@pytest.mark.gpu
@pytest.mark.parametrize("windows_per_launch", [1, 3])
def test_gpu_compact_block_files(ds, oracle, gpu_ctx, tmp_path, windows_per_launch):
    """real_compact from block files on disk through 8 MiB windows (FileIterator,
    logic_block.cpp:1132-1329; task.cpp:713-836): arbitrary sizes (every
    destination shift), two files larger than a window (write_big_file), files
    deleted and concealed through the index, a FileInfo that disagrees with its
    index entry (FI_INVALID, skipped), a corrupted live payload in an extension
    block (copied, reported -1010).  The new block files must hold exactly the
    oracle's real_compact output of the stitched source, and the new index the
    new metas and BlockInfo."""
    from test_gpu_parity import _oracle_compact
    rng = np.random.default_rng(1234)
    sizes = [int(x) for x in rng.integers(0, 300_000, 150)]
    sizes[20] = 9 * MiB + 77          # big files: more than one window each
    sizes[90] = 17 * MiB + 3
    sizes[5], sizes[6], sizes[7] = 0, 1, 35
    flags = {3: 1, 4: 1, 30: 1, 31: 4, 60: 5, 93: 1, 120: 1}
    blk = make_block(ds, oracle, 606, sizes, seed=7, flags=flags)
    main_size, ext_size = 16 * MiB, 8 * MiB
    src, dst = str(tmp_path / "src"), str(tmp_path / "dst")
    ds.write_block_files(blk, src, 12, 300, bucket_size=17, main_size=main_size, ext_size=ext_size)
    lb0 = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    m0 = lb0.metas
    # FileInfo id of file 50 rewritten on disk: index and header disagree -> FI_INVALID
    o50 = int(m0["offset"][np.nonzero(m0["file_id"] == 50)[0][0]])
    _flip_on_disk(src, lb0.chain, main_size, ext_size, o50, 0x01)
    # a live payload byte corrupted where it lies in an extension block
    k = next(i for i in range(len(m0)) if int(m0["offset"][i]) > main_size and int(m0["size"][i]) > 1000
             and int(m0["file_id"][i]) not in flags and int(m0["file_id"][i]) != 50)
    bad_id = int(m0["file_id"][k])
    _flip_on_disk(src, lb0.chain, main_size, ext_size, int(m0["offset"][k]) + 36 + 700)
    lb = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    img = lb.data()
    odest, doff, ook = _oracle_compact(oracle, img, lb.metas, lb.flags)
    live = np.nonzero((lb.flags & 3) == 0)[0]
    assert lb.flags[np.nonzero(lb.metas["file_id"] == 50)[0][0]] == 2
    rc, dmetas, st, ext, cnt = ds.compact_block_files(gpu_ctx, src, 12, dst, 40, 700, bucket_size=0,
                                                      windows_per_launch=windows_per_launch,
                                                      main_size=main_size, ext_size=ext_size)
    exp_st = np.where(ook[live] == 1, 0, -1010)
    assert cnt["n_live"] == len(live) and cnt["big_files"] == 2 and cnt["windows"] > 4, cnt
    assert np.array_equal(st, exp_st), (np.nonzero(st != exp_st)[0][:10], np.nonzero(exp_st)[0], cnt)
    assert rc == -1010 and cnt["n_bad"] == 1, (rc, cnt)
    assert cnt["dest_size"] == odest.size
    assert np.array_equal(dmetas["file_id"], lb.metas["file_id"][live])
    assert np.array_equal(dmetas["size"], lb.metas["size"][live])
    assert np.array_equal(dmetas["offset"].astype(np.int64), doff[live])
    assert int(st[list(dmetas["file_id"]).index(bad_id)]) == -1010
    out = ds.LoadedBlock(None, dst, 40, main_size=main_size, ext_size=ext_size)
    assert out.rc == 0 and out.logic_block_id == 606 and out.chain == [40] + ext
    assert np.array_equal(out.data(), odest)
    assert np.array_equal(out.metas, dmetas)
    h, h0 = out.header[0], lb.header[0]
    assert h["file_count"] == len(live) and h["size"] == odest.size and h["data_file_offset"] == odest.size
    assert h["del_file_count"] == 0 and h["del_size"] == 0 and h["version"] == h0["version"] + 1
    assert h["seq_no"] == h0["seq_no"] and h["bucket_size"] == 17
    # the concealed file keeps its flag in the new FileInfo; the corrupted one keeps its stored crc_
    assert out.flags[list(out.metas["file_id"]).index(31)] == 4
    # verify-on-read of the new block: the corrupted file fails its CRC; the empty
    # file (id 6) is rejected as the reference's sync_backup rejects it
    # (read length <= sizeof(FileInfo), sync_backup.cpp:348-351)
    rc2, st2 = ds.verify_block_files(gpu_ctx, dst, 40, main_size=main_size, ext_size=ext_size)
    ids = list(out.metas["file_id"])
    assert rc2 == 2 and st2[ids.index(bad_id)] == -1010 and st2[ids.index(6)] == -8034
    assert int((st2 != 0).sum()) == 2


@pytest.mark.gpu
def test_gpu_compactor_reused_across_blocks(ds, oracle, gpu_ctx, tmp_path):
    """One BlockFileCompactor (window buffers and streams kept) compacts three
    different blocks in turn, one of them with a file over a window and one with
    a corrupted payload; each new block equals the oracle's real_compact of its
    source, and a failed call (missing source) leaves the compactor usable."""
    from test_gpu_parity import _oracle_compact
    main_size, ext_size = 16 * MiB, 8 * MiB
    src, dst = str(tmp_path / "src"), str(tmp_path / "dst")
    comp = ds.BlockFileCompactor(gpu_ctx, windows_per_launch=2)
    rng = np.random.default_rng(99)
    try:
        for k in range(3):
            sizes = [int(x) for x in rng.integers(0, 200_000, 90 + 20 * k)]
            if k == 1:
                sizes[10] = 9 * MiB + 5
            flags = {int(i): 1 for i in rng.choice(len(sizes), 25, replace=False) + 1}
            blk = make_block(ds, oracle, 700 + k, sizes, seed=40 + k, flags=flags)
            ds.write_block_files(blk, src, 10 + k, 100 + 10 * k, bucket_size=31, main_size=main_size,
                                 ext_size=ext_size)
            lb0 = ds.LoadedBlock(None, src, 10 + k, main_size=main_size, ext_size=ext_size)
            bad_id = None
            if k == 2:
                m0 = lb0.metas
                j = next(i for i in range(len(m0)) if int(m0["size"][i]) > 1000 and int(m0["file_id"][i]) not in flags)
                bad_id = int(m0["file_id"][j])
                _flip_on_disk(src, lb0.chain, main_size, ext_size, int(m0["offset"][j]) + 36 + 500)
            lb = ds.LoadedBlock(None, src, 10 + k, main_size=main_size, ext_size=ext_size)
            odest, doff, ook = _oracle_compact(oracle, lb.data(), lb.metas, lb.flags)
            live = np.nonzero((lb.flags & 3) == 0)[0]
            rc, dmetas, st, ext, cnt = comp.compact(src, 10 + k, dst, 50 + k, 400 + 10 * k, main_size=main_size,
                                                    ext_size=ext_size)
            assert cnt["n_live"] == len(live) and cnt["dest_size"] == odest.size, (k, cnt)
            assert rc == (-1010 if k == 2 else 0) and cnt["n_bad"] == (1 if k == 2 else 0), (k, rc, cnt)
            assert cnt["big_files"] == (1 if k == 1 and 11 not in flags else 0), (k, cnt)
            assert np.array_equal(dmetas["offset"].astype(np.int64), doff[live])
            out = ds.LoadedBlock(None, dst, 50 + k, main_size=main_size, ext_size=ext_size)
            assert out.rc == 0 and np.array_equal(out.data(), odest), k
            if bad_id is not None:
                assert int(st[list(dmetas["file_id"]).index(bad_id)]) == -1010
        rc, _, _, _, _ = comp.compact(src, 99, dst, 90, 900, main_size=main_size, ext_size=ext_size)
        assert rc != 0
        rc, _, _, _, cnt = comp.compact(src, 10, dst, 91, 910, main_size=main_size, ext_size=ext_size)
        assert rc == 0 and cnt["n_live"] > 0
    finally:
        comp.free()


@pytest.mark.gpu
def test_gpu_compact_refuses_destination_in_source_chain(ds, oracle, gpu_ctx, tmp_path):
    """real_compact always writes another logic block.  A destination that is one
    of the source chain's files -- the same mount and main id, an extension id of
    the source chain, or the same files behind a symlinked mount -- would be
    truncated (O_TRUNC) before it is read: refused with EXIT_PARAMETER_ERROR and
    nothing written.  A different main id in the same mount works."""
    from test_gpu_parity import _oracle_compact
    rng = np.random.default_rng(808)
    sizes = [int(x) for x in rng.integers(0, 120_000, 40)]
    flags = {3: 1, 9: 1, 20: 4}
    blk = make_block(ds, oracle, 515, sizes, seed=81, flags=flags)
    main_size, ext_size = 1 * MiB, 512 * 1024
    src = str(tmp_path / "src")
    ext = ds.write_block_files(blk, src, 12, 300, bucket_size=7, main_size=main_size, ext_size=ext_size)
    assert len(ext) >= 2
    before = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    data0, metas0 = before.data(), before.metas.copy()
    link = str(tmp_path / "link")
    os.symlink(src, link)
    for dst, dst_id, first_ext in ((src, 12, 700), (src, 13, ext[1]), (src, 13, ext[0] - 3), (link, 12, 900),
                                   (link, 14, ext[0])):
        rc, _, _, _, _ = ds.compact_block_files(gpu_ctx, src, 12, dst, dst_id, first_ext, main_size=main_size,
                                                ext_size=ext_size)
        assert rc == -1016, (dst, dst_id, first_ext, rc)
        again = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
        assert again.rc == 0 and np.array_equal(again.data(), data0) and np.array_equal(again.metas, metas0)
    assert not os.path.exists(os.path.join(src, "13")) and not os.path.exists(os.path.join(src, "14"))
    rc, dmetas, st, ext2, cnt = ds.compact_block_files(gpu_ctx, src, 12, src, 13, 800, main_size=main_size,
                                                       ext_size=ext_size)
    assert rc == 0 and cnt["n_dropped"] == 0
    odest, doff, ook = _oracle_compact(oracle, data0, before.metas, before.flags)
    out = ds.LoadedBlock(None, src, 13, main_size=main_size, ext_size=ext_size)
    assert out.rc == 0 and np.array_equal(out.data(), odest)
    again = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    assert np.array_equal(again.data(), data0)


@pytest.mark.gpu
def test_gpu_compact_dropped_records_and_big_file_header(ds, oracle, gpu_ctx, tmp_path):
    """Two divergences of round 2 (ADVICE) pinned down:
    - a file over a window whose FileInfo disagrees with the index is copied, as
      the reference's big-file branch does (FileIterator, logic_block.cpp:
      1221-1240: no id/size check there; write_big_file, task.cpp:838-880);
    - a record that cannot be read whole (here: running past a data area
      declared 100 bytes short) is not copied and is reported (n_dropped).
      The reference would read past the declared end; no fixture covers it
      (parity unpinned), so the restatement reports it rather than guess."""
    from test_gpu_parity import _oracle_compact
    rng = np.random.default_rng(909)
    sizes = [int(x) for x in rng.integers(100, 150_000, 50)]
    sizes[10] = 9 * MiB + 11
    blk = make_block(ds, oracle, 616, sizes, seed=91)
    main_size, ext_size = 16 * MiB, 8 * MiB
    src, dst = str(tmp_path / "src"), str(tmp_path / "dst")
    ds.write_block_files(blk, src, 12, 300, bucket_size=11, main_size=main_size, ext_size=ext_size)
    lb0 = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    m0 = lb0.metas
    big = int(np.nonzero(m0["file_id"] == 11)[0][0])
    _flip_on_disk(src, lb0.chain, main_size, ext_size, int(m0["offset"][big]), 0x01)  # FileInfo id_ byte 0
    last = int(np.argmax(m0["offset"]))
    ipath = os.path.join(src, "index", "12")
    with open(ipath, "r+b") as f:
        f.seek(36)  # IndexHeader.data_file_offset_ (after 9 int32 fields)
        dfo = struct.unpack("<i", f.read(4))[0]
        f.seek(36)
        f.write(struct.pack("<i", dfo - 100))
    lb = ds.LoadedBlock(None, src, 12, main_size=main_size, ext_size=ext_size)
    assert lb.rc == 0 and lb.header[0]["data_file_offset"] == dfo - 100
    assert lb.flags[big] == 2  # the window path's FI_INVALID
    fl = lb.flags.copy()
    fl[big] = 0                # ... the big-file path copies it
    fl[last] = 2               # ... the truncated record is dropped
    odest, doff, ook = _oracle_compact(oracle, lb.data(), lb.metas, fl)
    rc, dmetas, st, ext, cnt = ds.compact_block_files(gpu_ctx, src, 12, dst, 40, 700, main_size=main_size,
                                                      ext_size=ext_size)
    assert rc == 0 and cnt["n_bad"] == 0, (rc, cnt)
    assert cnt["big_files"] == 1 and cnt["n_dropped"] == 1, cnt
    assert cnt["n_live"] == len(sizes) - 1
    assert int(m0["file_id"][last]) not in set(dmetas["file_id"].tolist())
    out = ds.LoadedBlock(None, dst, 40, main_size=main_size, ext_size=ext_size)
    assert out.rc == 0 and np.array_equal(out.data(), odest)


@pytest.mark.gpu
def test_pool_backed_block_stays_page_locked_and_pool_free_refused(ds, oracle, gpu_ctx):
    """A pooled LogicBlock takes its whole arena up front (appends never move it
    to pageable memory), its capacity is the arena's, the block keeps its pool
    alive, and the pool refuses to free arenas still lent to a block."""
    pool = ds.BlockImagePool(gpu_ctx, 2, 4 * MiB)
    try:
        assert pool.size() == 2 and pool.in_use() == 0
        b = ds.LogicBlock(5, capacity=1 << 40, pool=pool)
        assert b.pool is pool
        payload = synth_bytes(3, 60_000).tobytes()
        c = ocrc(oracle, 0, payload)
        n = 0
        while b.append(n + 1, payload, c) == 0:
            n += 1
        assert n == (4 * MiB) // (60_000 + 36)  # capacity capped at the arena, never grown past it
        assert pool.in_use() == 1
        with pytest.raises(RuntimeError):
            pool.free()
        nbad, st = ds.verify_block(gpu_ctx, b)
        assert nbad == 0 and len(st) == n
        b.free()
        assert pool.in_use() == 0
    finally:
        pool.free()
