"""Round-3 boundary checks on the GPU:

- the scalar Func::crc drop-in's failure mode (include/tfs_crc.h): a device
  error is counted and, through tfs_crc32_e, reported as TFS_CRC_EXIT_DEVICE_ERROR
  -- never as a CRC mismatch -- on the scalar path, the packet decode check
  (base_packet.cpp:141) and a sync_backup-shaped running CRC
  (sync_backup.cpp:383,412); the scalar context is selectable per process and
  per thread;
- scheduler slots on streams the context does not own (a caller's
  hipStream_t): any number of them, two in flight at once, each launch
  oracle-exact; hipStreamPerThread refused.
"""
import ctypes
import threading

import numpy as np
import pytest

from conftest import ocrc
from test_latency_form import _oracle_batch
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

DEVICE_ERROR = -20001
CHECK_CRC_ERROR = -1010


def _scalar_e(L, seed, data):
    err = ctypes.c_int(0)
    v = L.tfs_crc32_e(seed & 0xFFFFFFFF, data, len(data), ctypes.byref(err))
    return v, err.value


def test_scalar_device_error_is_counted_and_reported(oracle):
    import tfs_amd.crc as crc
    L = crc.lib()
    ctx = crc.Context(0)
    try:
        assert L.tfs_crc32_bind_thread(ctx.handle) == 0
        assert L.tfs_crc32_default_ctx() == ctx.handle.value
        data = synth_bytes(1600, 65536).tobytes()
        good = ocrc(oracle, 7, data)
        assert _scalar_e(L, 7, data) == (good, 0)
        before = L.tfs_crc32_error_count()
        ctx.inject_device_error(0, 1)
        assert _scalar_e(L, 7, data) == (7, DEVICE_ERROR)  # the seed back, and the error beside it
        assert L.tfs_crc32_error_count() == before + 1
        ctx.inject_device_error(0, 1)
        assert L.tfs_crc32(7, data, len(data)) == 7        # no error channel: counted, not silent
        assert L.tfs_crc32_error_count() == before + 2
        assert b"injected" in L.tfs_crc32_last_error(None)
        assert _scalar_e(L, 7, data) == (good, 0)
        assert L.tfs_crc32_error_count() == before + 2
    finally:
        L.tfs_crc32_bind_thread(None)
        ctx.close()


def test_scalar_context_selectable_per_process_and_thread(oracle):
    import tfs_amd.crc as crc
    L = crc.lib()
    a, b = crc.Context(0), crc.Context(0)
    try:
        data = synth_bytes(1601, 4096).tobytes()
        want = ocrc(oracle, 0, data)
        assert L.tfs_crc32_set_default_ctx(a.handle) == 0
        res = {}

        def worker(name, bind):
            if bind is not None:
                L.tfs_crc32_bind_thread(bind.handle)
            res[name] = (L.tfs_crc32_default_ctx(), [crc.func_crc(0, data) for _ in range(5)])
            L.tfs_crc32_bind_thread(None)

        t1 = threading.Thread(target=worker, args=("default", None))
        t2 = threading.Thread(target=worker, args=("bound", b))
        for t in (t1, t2):
            t.start()
        for t in (t1, t2):
            t.join()
        assert res["default"] == (a.handle.value, [want] * 5)
        assert res["bound"] == (b.handle.value, [want] * 5)
        assert a.resident_stats()[1] == 5 and b.resident_stats()[1] == 5
    finally:
        L.tfs_crc32_set_default_ctx(None)
        a.close()
        b.close()
    assert L.tfs_crc32_default_ctx() not in (None, 0)  # back to device 0's own default


def test_thread_binding_to_a_destroyed_context_is_dropped(oracle):
    """a context destroyed on another thread no longer leaves this
    thread's binding dangling -- the next scalar call finds it gone and runs on the
    process default; binding a context that is not live is refused."""
    import tfs_amd.crc as crc
    L = crc.lib()
    data = synth_bytes(1602, 65536).tobytes()
    want = ocrc(oracle, 3, data)
    a = crc.Context(0)
    stale = a.handle.value
    res = {}
    go, done = threading.Event(), threading.Event()

    def worker():
        L.tfs_crc32_bind_thread(a.handle)
        res["bound"] = (L.tfs_crc32_default_ctx(), crc.func_crc(3, data))
        go.set()
        done.wait(60)
        res["after"] = (L.tfs_crc32_default_ctx(), crc.func_crc(3, data), _scalar_e(L, 3, data))
        L.tfs_crc32_bind_thread(None)

    t = threading.Thread(target=worker)
    t.start()
    assert go.wait(60)
    a.close()  # destroyed on this thread while the worker is still bound to it
    done.set()
    t.join(120)
    assert res["bound"] == (stale, want)
    d, v, ve = res["after"]
    assert d not in (None, 0) and v == want and ve == (want, 0)
    assert L.tfs_crc32_bind_thread(ctypes.c_void_p(stale)) == -1016  # TFS_EXIT_PARAMETER_ERROR: not live


def test_packet_decode_device_error_is_not_a_crc_mismatch(oracle):
    """BasePacket::decode's CRC check (base_packet.cpp:141) through the batched
    receive path and the C++ PacketDecoder: an injected device error is -20001."""
    import test_packet as tp
    import tfs_amd.crc as crc
    import tfs_amd.dataserver as ds
    ctx = crc.Context(0)
    try:
        rng = np.random.default_rng(22)
        buf, frames, kinds = tp.build_stream(rng, n=20)
        offs, lens = [f[0] for f in frames], [f[1] for f in frames]
        crc_, st, nbad, rc = ctx.packet_verify(buf, offs, lens)
        assert rc in (0, CHECK_CRC_ERROR)
        ctx.inject_device_error(0, 1)
        with pytest.raises(crc.TfsCrcError) as e:
            ctx.packet_verify(buf, offs, lens)
        assert e.value.code == DEVICE_ERROR
        assert ctx.packet_verify(buf, offs, lens)[3] == rc  # and works again
        # the C++ PacketDecoder (packet_codec.cpp) over a connection's contiguous frames
        from tfs_amd import packet as pk
        import zlib
        frames_raw = []
        for i in range(12):
            body = pk.write_data_body(100 + i, 200 + i, 0, synth_bytes(1603 + i, 5000 + 97 * i).tobytes())
            c = (~zlib.crc32(body, ~pk.TFS_PACKET_FLAG_V1 & 0xFFFFFFFF)) & 0xFFFFFFFF  # Func::crc(FLAG_V1, body)
            frames_raw.append(pk.frame_v1(body, pid=i, crc=c))
        stream = b"".join(frames_raw)
        rc1, off1, st1, crc1, used1 = ds.decode_stream(ctx, stream)
        assert rc1 == 0 and len(st1) == 12 and (st1 == 0).all() and used1 == len(stream)
        ctx.inject_device_error(0, 1)
        rc2 = ds.decode_stream(ctx, stream)[0]
        assert rc2 == DEVICE_ERROR
        bad = bytearray(stream)
        bad[len(frames_raw[0]) + 40] ^= 1  # a body byte of frame 1: a real mismatch
        rc3, _, st3, _, _ = ds.decode_stream(ctx, bytes(bad))
        assert rc3 != DEVICE_ERROR and st3[1] == CHECK_CRC_ERROR and (np.delete(st3, 1) == 0).all()
    finally:
        ctx.close()


def _sync_backup_copy_check(L, data, stored_crc, chunk=1 << 20):
    """TfsMirrorBackup::copy_file's running check (sync_backup.cpp:383,412,429)
    with the scalar drop-in routed through tfs_crc32_e: a device
    error maps to -20001, a mismatch to EXIT_CHECK_CRC_ERROR (-1010)."""
    crc_ = 0
    for off in range(0, len(data), chunk):
        part = data[off:off + chunk]
        err = ctypes.c_int(0)
        crc_ = L.tfs_crc32_e(crc_, part, len(part), ctypes.byref(err))
        if err.value != 0:
            return DEVICE_ERROR
    return 0 if crc_ == stored_crc else CHECK_CRC_ERROR


def test_sync_backup_shaped_running_crc_device_error(oracle):
    import tfs_amd.crc as crc
    L = crc.lib()
    ctx = crc.Context(0)
    try:
        L.tfs_crc32_bind_thread(ctx.handle)
        data = synth_bytes(1602, 3 * (1 << 20) + 12345).tobytes()
        stored = ocrc(oracle, 0, data)
        assert _sync_backup_copy_check(L, data, stored) == 0
        assert _sync_backup_copy_check(L, data, stored ^ 1) == CHECK_CRC_ERROR
        ctx.inject_device_error(1, 1)  # the second 1 MiB chunk fails
        assert _sync_backup_copy_check(L, data, stored) == DEVICE_ERROR
        assert _sync_backup_copy_check(L, data, stored) == 0
    finally:
        L.tfs_crc32_bind_thread(None)
        ctx.close()


# ---- scheduler slots of caller-owned streams ---------------------------------

def _hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return h


def _device_files(ctx, oracle, n, seed, maxlen=200):
    import tfs_amd.crc as crc
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 5, n).astype(np.uint64))
    buf = synth_bytes(seed, int(offs[-1] + lens[-1]) + 64)
    exp = _oracle_batch(oracle, buf, offs, lens, np.zeros(n, np.uint32))
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, exp
    img = crc.DeviceBuffer(ctx, buf.size).upload(buf)
    dd = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
    return img, dd, exp


def test_caller_streams_any_number_and_concurrent(gpu_ctx, oracle):
    """300 hipStream_t of the caller's own (more than the 256 slots), each used
    for a dynamic-ticket verify and destroyed with hipStreamDestroy, never through
    the ABI; pairs in flight together on two such streams; every verdict of
    every launch checked.  The ctx binds no slot to them."""
    import tfs_amd.crc as crc
    hip = _hip()
    n = 70000  # >= 16 files per wave: dynamic tickets on the slot
    img, dd, exp = _device_files(gpu_ctx, oracle, n, 1700)
    outs = [crc.DeviceBuffer(gpu_ctx, n) for _ in range(2)]
    bads = [crc.DeviceBuffer(gpu_ctx, 4) for _ in range(2)]
    owned0, foreign0 = gpu_ctx.sched_stats()
    try:
        for it in range(150):
            ss = []
            for k in range(2):
                s = ctypes.c_void_p()
                assert hip.hipStreamCreate(ctypes.byref(s)) == 0
                ss.append(s.value)
            for k in range(2):
                outs[k].zero(stream=ss[k])
                bads[k].zero(stream=ss[k])
                gpu_ctx.verify_device(dd, n, img, None, outs[k], bads[k], stream=ss[k])
            for k in range(2):
                assert hip.hipStreamSynchronize(ss[k]) == 0
                assert int(bads[k].download(np.uint32)[0]) == 0, (it, k)
                if it % 25 == 0:
                    assert (outs[k].download(np.uint8, n) == 1).all(), (it, k)
                assert hip.hipStreamDestroy(ss[k]) == 0
        owned, foreign = gpu_ctx.sched_stats()
        assert owned == owned0 and foreign - foreign0 == 300
    finally:
        for b in outs + bads + [img, dd]:
            b.free()


def test_foreign_streams_share_one_split_plan(oracle):
    """Throughput launches on many streams of the caller's own (foreign slots) use
    ONE split plan between them: after 40 such launches on 40 streams,
    with files long enough to be split, the context holds one plan more than its
    owned streams' -- not one per foreign slot -- and every CRC is exact."""
    import tfs_amd.crc as crc
    hip = _hip()
    ctx = crc.Context(0)
    n = 3000
    rng = np.random.default_rng(1703)
    lens = np.where(rng.integers(0, 10, n) == 0, rng.integers(1 << 17, 1 << 19, n), rng.integers(0, 4000, n))
    lens = lens.astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64))
    buf = synth_bytes(1704, int(offs[-1] + lens[-1]) + 64)
    exp = _oracle_batch(oracle, buf, offs, lens, np.zeros(n, np.uint32))
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"] = offs, lens
    img = crc.DeviceBuffer(ctx, buf.size).upload(buf)
    dd = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
    outs = [crc.DeviceBuffer(ctx, 4 * n) for _ in range(4)]
    streams = []
    try:
        ctx.batch_device(dd, n, img, outs[0])  # the ctx stream's own plan
        ctx.sync()
        plans0, bytes0 = ctx.plan_stats()
        assert plans0 == 1
        for it in range(40):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            streams.append(s.value)
            ctx.batch_device(dd, n, img, outs[it % 4], stream=s.value)
            if it % 4 == 3:  # four launches in flight on four streams at a time
                for q in streams[-4:]:
                    assert hip.hipStreamSynchronize(q) == 0
                for k in range(4):
                    assert (outs[k].download(np.uint32, n) == exp).all(), (it, k)
        plans, nbytes = ctx.plan_stats()
        assert plans == plans0 + 1 and nbytes <= 2 * bytes0, (plans, nbytes, bytes0)
    finally:
        for q in streams:
            hip.hipStreamDestroy(q)
        for b in outs + [img, dd]:
            b.free()
        ctx.close()


def test_stream_per_thread_handle_refused(gpu_ctx, oracle):
    import tfs_amd.crc as crc
    img, dd, exp = _device_files(gpu_ctx, oracle, 100, 1701)
    try:
        with pytest.raises(crc.TfsCrcError) as e:
            gpu_ctx.verify_device(dd, 100, img, stream=2)  # hipStreamPerThread
        assert e.value.code == crc.TFS_EXIT_PARAMETER_ERROR and "PerThread" in str(e.value)
    finally:
        img.free()
        dd.free()


def test_owned_streams_keep_their_slots(gpu_ctx, oracle):
    """Streams made by tfs_crc32_stream_create own a slot each (no per-launch
    memset); destroying one frees its slot for the next."""
    import tfs_amd.crc as crc
    n = 70000
    img, dd, exp = _device_files(gpu_ctx, oracle, n, 1702)
    out = crc.DeviceBuffer(gpu_ctx, 4 * n)
    ok = crc.DeviceBuffer(gpu_ctx, n)
    bad = crc.DeviceBuffer(gpu_ctx, 4)
    owned0, foreign0 = gpu_ctx.sched_stats()
    try:
        for it in range(20):
            st = gpu_ctx.stream_create()
            assert gpu_ctx.sched_stats()[0] == owned0 + 1
            ok.zero(stream=st)
            bad.zero(stream=st)
            for _ in range(3):
                gpu_ctx.verify_device(dd, n, img, out, ok, bad, stream=st)
            gpu_ctx.stream_sync(st)
            assert (out.download(np.uint32, n) == exp).all(), it
            assert (ok.download(np.uint8, n) == 1).all() and int(bad.download(np.uint32)[0]) == 0, it
            gpu_ctx.stream_destroy(st)
        assert gpu_ctx.sched_stats() == (owned0, foreign0)
    finally:
        for b in (out, ok, bad, img, dd):
            b.free()


def test_stats_count_lone_small_calls(oracle):
    """tfs_crc32_stats: every synchronous host call is counted,
    and the lone ones (one body) under TFS_CRC_LONE_CROSSOVER bytes -- the calls
    an integration should batch -- separately with their bytes, the scalar
    drop-in's included (on the context it runs on); the results stay exact."""
    import tfs_amd.crc as crc
    L = crc.lib()
    ctx = crc.Context(0)
    try:
        buf = synth_bytes(77, 3 * crc.LONE_CROSSOVER)
        raw = buf.tobytes()
        s0 = ctx.stats()
        assert all(v == 0 for v in s0.values()), s0
        assert ctx.batch(buf, [5], [100])[0] == ocrc(oracle, 0, raw[5:105])              # lone, small
        n = crc.LONE_CROSSOVER
        assert ctx.batch(buf, [0], [n])[0] == ocrc(oracle, 0, raw[:n])                  # lone, at the crossover
        assert ctx.batch(buf, [0], [n - 1])[0] == ocrc(oracle, 0, raw[:n - 1])          # lone, just under
        got = ctx.batch(buf, [0, 300, 900], [10, 20, 30])                               # three bodies
        assert [int(x) for x in got] == [ocrc(oracle, 0, raw[o:o + k]) for o, k in ((0, 10), (300, 20), (900, 30))]
        exp = ocrc(oracle, 0, raw[7:7 + 64])
        _, ok, nbad, rc = ctx.verify(buf, [7], [64], [exp])                            # lone verify, small
        assert nbad == 0 and ok[0] == 1
        assert L.tfs_crc32_bind_thread(ctx.handle) == 0
        try:
            assert L.tfs_crc32(0, raw[:33], 33) == ocrc(oracle, 0, raw[:33])            # scalar, small
        finally:
            L.tfs_crc32_bind_thread(None)
        s1 = ctx.stats()
        assert s1["host_calls"] == 6 and s1["host_files"] == 8, s1
        assert s1["lone_calls"] == 5, s1
        assert s1["lone_small_calls"] == 4 and s1["lone_small_bytes"] == 100 + (n - 1) + 64 + 33, s1
        assert s1["resident_files"] >= 0 and s1["resident_ring_full"] == 0
    finally:
        ctx.close()
