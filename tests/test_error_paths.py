"""Error paths at the drop-in boundary (VERDICT r1 "fix the boundary error path"):
a device failure surfaces as TFS_CRC_EXIT_DEVICE_ERROR (-20001) -- never as a
CRC value that the close path would compare and report as client corruption
(EXIT_DATA_FILE_ERROR, data_management.cpp:196-198) -- and nothing is
persisted; a partially computed spill CRC is never cached; capacity is checked
the same way for batched and unbatched closes.  Device failures are injected
through the C ABI (tfs_crc32_inject_device_error)."""
import numpy as np
import pytest

import tfs_amd.crc as crc_mod
from conftest import ocrc
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

DEVICE_ERROR = -20001
BLOCK_EXHAUST = -8004   # EXIT_BLOCK_EXHAUST_ERROR, error_msg.h:140


@pytest.fixture(scope="module")
def ds():
    import tfs_amd.dataserver as ds
    ds.lib()
    return ds


@pytest.fixture
def ctx():
    c = crc_mod.Context(0)
    yield c
    c.close()


def test_close_device_error_persists_nothing(ctx, ds, oracle, tmp_path):
    data = synth_bytes(1, 70000).tobytes()
    client = ocrc(oracle, 0, data)
    df = ds.DataFile(ctx, 1, str(tmp_path))
    df.set_data(data, 0)
    blk = ds.LogicBlock(10)
    ctx.inject_device_error(0, 1)
    assert blk.close_write_file(1, client, df) == DEVICE_ERROR     # not -8013
    assert blk.raw().size == 0 and len(blk.metas()[0]) == 0
    # the lease is intact: the next close computes the CRC afresh and persists
    assert blk.close_write_file(1, client, df) == 0
    m, _ = blk.metas()
    assert len(m) == 1 and int(m["size"][0]) == len(data) + 36


def test_spill_crc_device_error_midway_is_not_cached(ctx, ds, oracle, tmp_path):
    """> 2 MiB: the chunked re-read (data_file.cpp:172-187) fails on its second chunk;
    get_crc reports the device error and a later call returns the full CRC, not
    the running value of the first chunk."""
    data = synth_bytes(2, 5 * (1 << 20) + 123).tobytes()
    df = ds.DataFile(ctx, 2, str(tmp_path))
    df.set_data(data, 0)
    ctx.inject_device_error(1, 1)
    with pytest.raises(crc_mod.TfsCrcError) as e:
        df.get_crc()
    assert e.value.code == DEVICE_ERROR
    try:
        got = df.get_crc()
    except crc_mod.TfsCrcError as e2:
        raise AssertionError((e2.code, crc_mod.lib().tfs_crc32_last_error(ctx.handle), ctx.resident_stats()))
    assert got == ocrc(oracle, 0, data)


def test_batched_close_device_error(ctx, ds, oracle, tmp_path):
    data = synth_bytes(3, 65536).tobytes()
    client = ocrc(oracle, 0, data)
    b = ds.CloseBatcher(ctx, max_batch=1, max_wait_us=50)
    try:
        df = ds.DataFile(ctx, 3, str(tmp_path))
        df.set_data(data, 0)
        blk = ds.LogicBlock(11)
        ctx.inject_device_error(0, 1)
        assert b.close(blk, 3, client, df) == DEVICE_ERROR
        assert blk.raw().size == 0
        assert b.close(blk, 3, client, df) == 0
        assert b.close(blk, 4, client ^ 1, df) == -8013               # a real mismatch still is one
        assert len(blk.metas()[0]) == 1
    finally:
        b.free()


def test_capacity_checked_for_batched_and_unbatched_closes(ctx, ds, oracle, tmp_path):
    """A block with room for three 1000-byte records: the fourth close fails with
    EXIT_BLOCK_EXHAUST_ERROR on both paths and leaves the block as it was."""
    data = synth_bytes(4, 1000).tobytes()
    client = ocrc(oracle, 0, data)
    b = ds.CloseBatcher(ctx, max_batch=1, max_wait_us=50)
    try:
        for batched in (False, True):
            blk = ds.LogicBlock(12, capacity=3 * (1000 + 36))
            rcs = []
            for fid in range(1, 5):
                df = ds.DataFile(ctx, fid, str(tmp_path))
                df.set_data(data, 0)
                rcs.append(b.close(blk, fid, client, df) if batched else blk.close_write_file(fid, client, df))
                df.free()
            assert rcs == [0, 0, 0, BLOCK_EXHAUST], batched
            assert blk.raw().size == 3 * 1036 and len(blk.metas()[0]) == 3
    finally:
        b.free()


def test_integration_sync_backup_shaped_verify(ctx, ds, oracle, tmp_path):
    """The verify-on-read binding INTEGRATION.md shows for sync_backup.cpp:383-429:
    FileInfo.size_ includes the 36-byte header (logic_block.cpp:173), so the
    payload descriptor is {FILEINFO_SIZE, size_ - FILEINFO_SIZE, crc_} over the
    bytes actually read."""
    data = synth_bytes(5, 123457).tobytes()
    df = ds.DataFile(ctx, 5, str(tmp_path))
    df.set_data(data, 0)
    blk = ds.LogicBlock(13)
    assert blk.close_write_file(5, ocrc(oracle, 0, data), df) == 0
    rc, rec = blk.read_file(5, len(data) + 36)               # FileInfo|payload, the read of :345-357
    assert rc == 0 and len(rec) == len(data) + 36
    fi = np.frombuffer(rec[:36], crc_mod.FILEINFO_DTYPE)[0]
    assert int(fi["size_"]) == len(data) + 36
    buf = np.frombuffer(rec, np.uint8)
    c, ok, nbad, rc = ctx.verify(buf, [36], [int(fi["size_"]) - 36], [int(fi["crc_"])])
    assert rc == 0 and nbad == 0 and int(c[0]) == ocrc(oracle, 0, data)
    bad = bytearray(rec)
    bad[36 + 1000] ^= 4
    c, ok, nbad, rc = ctx.verify(np.frombuffer(bytes(bad), np.uint8), [36], [int(fi["size_"]) - 36],
                                 [int(fi["crc_"])])
    assert rc == -1010 and nbad == 1 and ok[0] == 0
    # the descriptor the advisor flagged (size_ as the payload length) overruns the record
    with pytest.raises(crc_mod.TfsCrcError) as e:
        ctx.verify(buf, [36], [int(fi["size_"])], [int(fi["crc_"])])
    assert e.value.code == -1016


def test_host_block_paths_report_injected_errors(ctx, oracle):
    """tfs_block_verify and tfs_blocks_compact surface the device error too."""
    from test_gpu_parity import _block_image
    img, metas = _block_image(oracle, [65536] * 4 + [100], seed=9)
    ctx.inject_device_error(0, 1)
    with pytest.raises(crc_mod.TfsCrcError) as e:
        ctx.block_verify(img, metas)
    assert e.value.code == DEVICE_ERROR
    assert ctx.block_verify(img, metas)[2] == 0
    ctx.inject_device_error(0, 1)
    with pytest.raises(crc_mod.TfsCrcError) as e:
        ctx.block_compact(img, metas, np.zeros(len(metas), np.int32))
    assert e.value.code == DEVICE_ERROR
