"""The dataserver-shaped C++ harness (tfs_amd/ds) driven the way the reference's
own gtest programs drive LogicBlock/DataFile directly
(tests/dataserver/test_logic_block_and_compact.cpp, test_sync_mirror.cpp).
Every CRC goes through the C ABI onto the GPU; expected values come from the
oracle (test infrastructure)."""
import threading

import numpy as np
import pytest

from conftest import ocrc
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

DATA_LENGTH = 4096             # int32 elements per small file (test_logic_block_and_compact.cpp)
MAX_COMPACT_READ_SIZE = 8388608  # dataserver_define.h:41
FILEINFO = 36


@pytest.fixture(scope="module")
def ds():
    import tfs_amd.dataserver as ds
    ds.lib()
    return ds


def _file_info(raw, off):
    import tfs_amd.crc as crc
    return np.frombuffer(raw[off:off + FILEINFO].tobytes(), crc.FILEINFO_DTYPE)[0]


def test_write_file_header_and_crc(gpu_ctx, ds, oracle, tmp_path):
    """testWriteFile (:194-247): data[i] = i, crc = get_crc(), close, FileInfo fields."""
    data = np.arange(DATA_LENGTH, dtype=np.int32).tobytes()
    df = ds.DataFile(gpu_ctx, 1, str(tmp_path))
    assert df.set_data(data, 0) == len(data)
    crc = df.get_crc()
    assert crc == ocrc(oracle, 0, data)
    blk = ds.LogicBlock(100)
    assert blk.close_write_file(1, crc, df) == 0
    raw = blk.raw()
    fi = _file_info(raw, 0)
    assert fi["id_"] == 1 and fi["offset_"] == 0 and fi["flag_"] == 0
    assert fi["size_"] == FILEINFO + DATA_LENGTH * 4 and fi["usize_"] == fi["size_"]
    assert fi["crc_"] == crc
    assert raw[FILEINFO:].tobytes() == data


def test_close_rejects_wrong_client_crc(gpu_ctx, ds, tmp_path):
    """data_management.cpp:197-198: client crc != DataFile crc -> EXIT_DATA_FILE_ERROR, nothing persisted."""
    df = ds.DataFile(gpu_ctx, 2, str(tmp_path))
    df.set_data(b"x" * 1000, 0)
    blk = ds.LogicBlock(101)
    assert blk.close_write_file(2, df.get_crc() ^ 1, df) == -8013
    assert blk.raw().size == 0


def test_datafile_spill_chunked_crc(gpu_ctx, ds, oracle, tmp_path, golden):
    """> 2 MiB: the tmp-file spill and the 2 MiB chunked get_crc with running seed (data_file.cpp:172-187)."""
    for v in golden["datafile_big"]:
        d = synth_bytes(v["gen"]["seed"], v["gen"]["len"]).tobytes()
        df = ds.DataFile(gpu_ctx, 77, str(tmp_path))
        # written in 3 fragments, out of order, like WriteDataMessage segments
        n = len(d)
        cuts = [0, n // 3, 2 * n // 3, n]
        for a, b in [(cuts[1], cuts[2]), (cuts[0], cuts[1]), (cuts[2], cuts[3])]:
            assert df.set_data(d[a:b], a) == b - a
        assert df.get_length() == n
        assert df.get_crc() == v["expected"]
        df.free()


def test_sync_mirror_1mib_printable(gpu_ctx, ds, oracle, tmp_path):
    """test_sync_mirror.cpp:185-270: 1 MiB random printable payload, client crc = Func::crc."""
    rng = np.random.default_rng(185)
    d = rng.integers(32, 127, 1 << 20, dtype=np.uint8).tobytes()
    client = ocrc(oracle, 0, d)
    df = ds.DataFile(gpu_ctx, 9, str(tmp_path))
    df.set_data(d, 0)
    blk = ds.LogicBlock(7)
    assert blk.close_write_file(9, client, df) == 0
    nbad, st = ds.verify_block(gpu_ctx, blk)
    assert nbad == 0 and (st == 0).all()


def test_complex_compact(gpu_ctx, ds, oracle, tmp_path):
    """testComplexCompact (:904-1021): 1000 files (3 big ones), delete evens, insert 500,
    delete every 3rd, compact; check order, FileInfo and contents -- plus the added
    re-CRC verify of every live file."""
    N = 1000
    src = ds.LogicBlock(300)
    ids = []
    next_id = [1]

    def write(i_big):
        fid = next_id[0]
        next_id[0] += 1
        if i_big:
            payload = synth_bytes(fid, MAX_COMPACT_READ_SIZE + 1).tobytes()
        else:
            j = np.arange(DATA_LENGTH, dtype=np.int64)
            payload = ((j + fid * j) & 0xFFFFFFFF).astype(np.uint32).tobytes()
        df = ds.DataFile(gpu_ctx, fid, str(tmp_path))
        df.set_data(payload, 0)
        crc = df.get_crc()
        assert src.close_write_file(fid, crc, df) == 0
        df.free()
        return fid

    for i in range(N):
        ids.append(write(i in (5, 200, 500)))
    for i in range(0, N, 2):
        assert src.set_flag(ids[i], 1) == 0          # unlink_file(DELETE) -> FI_DELETED
    ids = [ids[i] for i in range(1, N, 2)]
    for i in range(N // 2, N):
        ids.append(write(False))
    for i in range(0, N, 3):
        assert src.set_flag(ids[i], 1) == 0
    dest = ds.LogicBlock(301)
    rc, ok = ds.compact_block(gpu_ctx, src, dest)
    assert rc == 0
    m, f = src.metas()
    live_src = [(int(x["file_id"]), int(x["size"])) for x, fl in zip(m, f) if not fl & 3]
    assert (ok[(f & 3) == 0] == 1).all() and (ok[(f & 3) != 0] == 2).all()
    raw = dest.raw()
    dm, _ = dest.metas()
    expected_ids = [ids[i] for i in range(N) if i % 3 != 0]
    assert [int(x) for x in dm["file_id"]] == expected_ids == [a for a, _ in live_src]
    off = 0
    for k, fid in enumerate(expected_ids):
        fi = _file_info(raw, off)
        assert fi["id_"] == fid and fi["offset_"] == off
        assert fi["size_"] == fi["usize_"] == live_src[k][1]
        pay = raw[off + FILEINFO:off + fi["size_"]]
        if fi["size_"] - FILEINFO == DATA_LENGTH * 4:
            j = np.arange(DATA_LENGTH, dtype=np.int64)
            assert (pay.view(np.uint32) == ((j + fid * j) & 0xFFFFFFFF).astype(np.uint32)).all()
        assert fi["crc_"] == ocrc(oracle, 0, pay.tobytes())
        off += int(fi["size_"])
    assert off == raw.size
    # the compacted block verifies clean
    nbad, st = ds.verify_block(gpu_ctx, dest)
    assert nbad == 0


def test_batched_closes_from_threads(gpu_ctx, ds, oracle, tmp_path):
    """Concurrent leases closing through one CloseBatcher: one GPU verify per batch;
    wrong client CRCs get EXIT_DATA_FILE_ERROR, the rest are persisted."""
    blk = ds.LogicBlock(500)
    batcher = ds.CloseBatcher(gpu_ctx, max_batch=32, max_wait_us=500)
    nthreads, per = 8, 40
    results = {}
    lock = threading.Lock()

    def worker(t):
        for k in range(per):
            fid = 1 + t * per + k
            d = synth_bytes(fid, 1000 + 37 * k + t).tobytes()
            df = ds.DataFile(gpu_ctx, fid, str(tmp_path))
            df.set_data(d, 0)
            client = ocrc(oracle, 0, d)
            if fid % 13 == 0:
                client ^= 0x80000000
            rc = batcher.close(blk, fid, client, df)
            with lock:
                results[fid] = (rc, fid % 13 == 0)
            df.free()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert len(results) == nthreads * per
    for fid, (rc, bad) in results.items():
        assert rc == (-8013 if bad else 0), fid
    assert batcher.batches() < nthreads * per       # closes were actually batched
    m, _ = blk.metas()
    assert len(m) == sum(1 for rc, bad in results.values() if not bad)
    nbad, st = ds.verify_block(gpu_ctx, blk)
    assert nbad == 0
    batcher.free()


@pytest.mark.parametrize("max_batch", [1, 4])
def test_pooled_leases_checked_in_place(gpu_ctx, ds, oracle, tmp_path, max_batch):
    """Leases whose DataFile buffers come from a page-locked LeaseBufferPool close
    through a CloseBatcher on that pool with no gather copy (each member's payload
    checked where set_data put it, the batch spread over the pool).  Wrong client
    CRCs get -8013, the rest are persisted byte for byte; leases past the pool's
    size take heap buffers and the unbatched close, with the same verdicts; a spill
    (> 2 MiB) lease from the pool is checked from its tmp file; every buffer is back
    in the pool at the end."""
    pool = ds.LeaseBufferPool(gpu_ctx, 6)  # fewer buffers than 8 threads: some leases fall back to the heap
    batcher = ds.CloseBatcher(gpu_ctx, max_batch=max_batch, max_wait_us=300, pool=pool)
    blk = ds.LogicBlock(510)
    nthreads, per = 8, 30
    results, pooled = {}, []
    lock = threading.Lock()

    def worker(t):
        for k in range(per):
            fid = 1 + t * per + k
            d = synth_bytes(fid * 7, 3000 + 911 * k + 13 * t).tobytes()
            df = ds.DataFile(gpu_ctx, fid, str(tmp_path), pool=pool)
            df.set_data(d, 0)
            client = ocrc(oracle, 0, d)
            if fid % 11 == 0:
                client ^= 0x4
            rc = batcher.close(blk, fid, client, df)
            with lock:
                results[fid] = (rc, fid % 11 == 0, d)
                pooled.append(df.pooled())
            df.free()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert len(results) == nthreads * per and any(pooled)
    for fid, (rc, bad, _) in results.items():
        assert rc == (-8013 if bad else 0), fid
    m, _ = blk.metas()
    assert len(m) == sum(1 for rc, bad, _ in results.values() if not bad)
    raw = blk.raw()
    for rec in m:
        fid = int(rec["file_id"])
        d = results[fid][2]
        o = int(rec["offset"])
        assert raw[o + FILEINFO:o + FILEINFO + len(d)].tobytes() == d
        assert _file_info(raw, o)["crc_"] == ocrc(oracle, 0, d)
    nbad, _ = ds.verify_block(gpu_ctx, blk)
    assert nbad == 0
    # a spill lease from the pool (> 2 MiB): re-read from its tmp file in 2 MiB chunks
    big = synth_bytes(4242, (2 << 20) + 12345).tobytes()
    df = ds.DataFile(gpu_ctx, 9999, str(tmp_path), pool=pool)
    df.set_data(big, 0)
    assert batcher.close(blk, 9999, ocrc(oracle, 0, big), df) == 0
    assert pool.in_use() == 1
    with pytest.raises(RuntimeError):
        pool.free()  # refused while a DataFile holds a buffer
    df.free()
    assert pool.in_use() == 0
    batcher.free()
    blk.free()
    pool.free()


def test_verify_block_crc_errors_drive_repair(gpu_ctx, ds, oracle, tmp_path):
    """Verify-on-read finds corrupted payloads; BlockChecker counts crc_error_ per
    block and asks for repair at max_crc_error_nums (default 4, parameter.cpp:256)."""
    blk = ds.LogicBlock(600)
    for fid in range(1, 21):
        d = synth_bytes(fid, 65536).tobytes()
        df = ds.DataFile(gpu_ctx, fid, str(tmp_path))
        df.set_data(d, 0)
        assert blk.close_write_file(fid, ocrc(oracle, 0, d), df) == 0
        df.free()
    checker = ds.BlockCrcChecker(4)
    m, _ = blk.metas()
    for k in (2, 7, 11):
        blk.corrupt(int(m[k]["offset"]) + FILEINFO + 1000 * k, 0x10)
    nbad, st = ds.verify_block(gpu_ctx, blk, checker)
    assert nbad == 3 and [int(i) for i in np.nonzero(st)[0]] == [2, 7, 11]
    assert checker.errors(600) == 3 and not checker.needs_repair(600)
    blk.corrupt(int(m[15]["offset"]) + FILEINFO, 0x01)
    nbad, st = ds.verify_block(gpu_ctx, blk, checker)
    assert nbad == 4 and checker.needs_repair(600)
    checker.free()


def test_loopback_block_like_config1(gpu_ctx, ds, oracle):
    """BASELINE configs[0] through the harness (tfs_ds_loopback_block): worker
    threads stage and close every file through the CloseBatcher, then the block
    is verified.  Files whose client CRC is wrong are rejected (-8013) and not
    persisted; every persisted record equals FileInfo{crc_ = Func::crc(0, payload)}
    followed by the payload, as the oracle's loopback writes it."""
    n, L = 96, 4096 + 13
    pay = synth_bytes(0xC0F1, n * L)
    client = np.array([ocrc(oracle, 0, pay[i * L:(i + 1) * L].tobytes()) for i in range(n)], np.uint32)
    wrong = [3, 40, 95]
    client[wrong] ^= 0x10
    blk = ds.LogicBlock(7)
    bad = ds.loopback_block(gpu_ctx, pay, n, L, client, 8, blk)
    assert bad == len(wrong)
    metas, flags = blk.metas()
    assert sorted(int(x) for x in metas["file_id"]) == [i + 1 for i in range(n) if i not in wrong]
    raw = blk.raw()
    for m in metas:
        i = int(m["file_id"]) - 1
        fi = _file_info(raw, int(m["offset"]))
        assert fi["id_"] == i + 1 and fi["size_"] == L + FILEINFO and fi["offset_"] == int(m["offset"])
        assert fi["crc_"] == client[i]
        assert raw[int(m["offset"]) + FILEINFO:int(m["offset"]) + FILEINFO + L].tobytes() == pay[i * L:(i + 1) * L].tobytes()
    blk.free()


def test_recombine_block_skips_bad_crc(gpu_ctx, ds, oracle):
    """TranBlock::recombine_data (tools/transfer/block_console.cpp:502-613): deleted and
    invalid files are skipped, a FileInfo that disagrees with the index is skipped (:543),
    a payload whose CRC != crc_ is skipped (:569-577), concealed files are kept with their
    flag, and the survivors are repacked with offsets rewritten."""
    src = ds.LogicBlock(900)
    rng = np.random.default_rng(902)
    pays = {}
    for fid in range(1, 21):
        p = rng.integers(0, 256, int(rng.integers(0, 70000)), dtype=np.uint8).tobytes()
        pays[fid] = p
        assert src.append(fid, p, ocrc(oracle, 0, p)) == 0
    m, _ = src.metas()
    off = {int(x["file_id"]): int(x["offset"]) for x in m}
    assert src.set_flag(3, 1) == 0          # FI_DELETED
    assert src.set_flag(4, 2) == 0          # FI_INVALID
    assert src.set_flag(5, 4) == 0          # FI_CONCEAL: kept
    big = [f for f in (7, 11, 16) if len(pays[f]) > 0]
    for f in big:                           # payload corruption -> skipped for its CRC
        src.corrupt(off[f] + FILEINFO + len(pays[f]) // 2, 0x20)
    src.corrupt(off[9], 0x01)               # FileInfo id_ disagrees with the index
    dest = ds.LogicBlock(901)
    rc, nskip = ds.recombine_block(gpu_ctx, src, dest)
    assert rc == 0 and nskip == len(big)
    keep = [f for f in range(1, 21) if f not in (3, 4, 9) and f not in big]
    dm, df = dest.metas()
    assert [int(x) for x in dm["file_id"]] == keep
    assert [int(x) for x in df] == [4 if f == 5 else 0 for f in keep]
    raw = dest.raw()
    o = 0
    for f in keep:
        fi = _file_info(raw, o)
        assert fi["id_"] == f and fi["offset_"] == o and fi["size_"] == FILEINFO + len(pays[f])
        assert fi["flag_"] == (4 if f == 5 else 0)      # new_info.flag_ = finfo.flag_ (:587)
        assert raw[o + FILEINFO:o + fi["size_"]].tobytes() == pays[f]
        assert fi["crc_"] == ocrc(oracle, 0, pays[f])
        o += int(fi["size_"])
    assert o == raw.size
    nbad, _ = ds.verify_block(gpu_ctx, dest)
    assert nbad == 0
