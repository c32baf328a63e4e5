"""The resident form: synchronous small batches taken by a
kernel that stays on the GPU, from a page-locked ring, instead of a launch per
batch.  Every output is checked against the oracle; the stats show the ring was
used (and, with short idle/lifetime limits, that the kernel was relaunched)."""
import threading
import time

import numpy as np
import pytest

from conftest import ocrc
from test_latency_form import _oracle_batch
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, **env):
    import tfs_amd.crc as crc
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    ctx = crc.Context(0)
    for k in env:
        monkeypatch.delenv(k)
    return ctx


def _random_batch(rng, n, maxlen=70000, seed=0):
    lens = rng.integers(0, maxlen, n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 9, n).astype(np.uint64))
    buf = synth_bytes(seed, int(offs[-1] + lens[-1]) + 64)
    return buf, offs, lens


def test_resident_batches_match_oracle(monkeypatch, oracle):
    """Compute with seeds and verify (with mismatches) through the ring, batch sizes
    1..256, pageable and page-locked; the same calls with the ring off agree.  The
    batches that read more than 1 MiB over PCIe (bodies over 80 bytes; the shorter
    ones travel in the ring unit) take the bulk form: fence, non-temporal stripes."""
    import tfs_amd.crc as crc
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1)
    try:
        rng = np.random.default_rng(31)
        ring_files = bulk = 0
        for it, n in enumerate((1, 2, 3, 8, 17, 64, 200, 256)):
            buf, offs, lens = _random_batch(rng, n, maxlen=70000 if n <= 64 else 30000, seed=500 + n)
            ring_files += 3 * n  # spans <= 8 MiB: read in place, so through the ring
            bulk += int(lens[lens > 80].sum()) > 1 << 20
            seeds = rng.integers(0, 2**32, n).astype(np.uint32)
            exp = _oracle_batch(oracle, buf, offs, lens, seeds)
            assert (ctx.batch(buf, offs, lens, seeds) == exp).all(), n
            zexp = _oracle_batch(oracle, buf, offs, lens, np.zeros(n, np.uint32))
            want = zexp.copy()
            flip = rng.integers(0, n)
            want[flip] ^= 0x10
            c, ok, nbad, rc = ctx.verify(buf, offs, lens, want)
            assert (c == zexp).all() and nbad == 1 and rc == -1010 and int(np.argmin(ok)) == flip, n
            pin = crc.PinnedBuffer(ctx, buf.size)
            try:
                pin.array[:] = buf
                assert (ctx.batch(pin.array, offs, lens, seeds) == exp).all(), n
            finally:
                pin.free()
        launches, files = ctx.resident_stats()
        assert launches >= 1 and files == ring_files and bulk >= 2, (launches, files, ring_files, bulk)
        ctx.set_resident(False)
        buf, offs, lens = _random_batch(rng, 40, seed=77)
        seeds = rng.integers(0, 2**32, 40).astype(np.uint32)
        assert (ctx.batch(buf, offs, lens, seeds) == _oracle_batch(oracle, buf, offs, lens, seeds)).all()
        assert ctx.resident_stats()[1] == files  # the ring was not used
    finally:
        ctx.close()


def test_resident_idle_exit_and_relaunch(monkeypatch, oracle):
    """The kernel leaves after its idle time; the next batch relaunches it."""
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1, TFS_CRC_RESIDENT_IDLE_US=50)
    try:
        rng = np.random.default_rng(32)
        for it in range(12):
            buf, offs, lens = _random_batch(rng, 4, seed=600 + it)
            seeds = rng.integers(0, 2**32, 4).astype(np.uint32)
            assert (ctx.batch(buf, offs, lens, seeds) == _oracle_batch(oracle, buf, offs, lens, seeds)).all(), it
            time.sleep(0.003)
        launches, files = ctx.resident_stats()
        assert files == 48 and launches >= 6, (launches, files)
    finally:
        ctx.close()


@pytest.mark.parametrize("life_us", [10000, 300])
def test_resident_concurrent_threads(monkeypatch, oracle, life_us):
    """8 threads of synchronous verifies (1-8 files each, one wrong expected CRC per
    call) in flight together; with a 300 us lifetime the kernel is relaunched many
    times under load.  Every CRC and verdict of every call is checked."""
    import tfs_amd.crc as crc
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1, TFS_CRC_RESIDENT_LIFE_US=life_us)
    errors = []
    nthreads, calls = 8, 150
    try:
        pins = [crc.PinnedBuffer(ctx, 8 * 65536 + 64) for _ in range(nthreads)]

        def worker(t):
            try:
                rng = np.random.default_rng(1000 + t)
                pin = pins[t]
                for it in range(calls):
                    n = int(rng.integers(1, 9))
                    lens = rng.integers(0, 65536, n).astype(np.uint32)
                    offs = np.arange(n, dtype=np.uint64) * 65536 + rng.integers(0, 8, n).astype(np.uint64)
                    pin.array[:] = rng.integers(0, 256, pin.array.size, dtype=np.uint8)
                    exp = _oracle_batch(oracle, pin.array, offs, lens, np.zeros(n, np.uint32))
                    want = exp.copy()
                    flip = it % n
                    want[flip] ^= 1
                    c, ok, nbad, rc = ctx.verify(pin.array, offs, lens, want)
                    if not ((c == exp).all() and nbad == 1 and rc == -1010 and int(np.argmin(ok)) == flip):
                        errors.append((t, it, n))
                        return
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        launches, files = ctx.resident_stats()
        for p in pins:
            p.free()
    finally:
        ctx.close()
    assert not errors, errors[:5]
    assert files > 0
    if life_us == 300:
        assert launches > 2, launches


def test_resident_scalar_drop_in(oracle):
    """tfs_crc32 (the Func::crc drop-in, default context) goes through the ring."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(33)
    for it in range(300):
        n = int(rng.integers(0, 70000))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert crc.func_crc(s, d) == ocrc(oracle, s, d), it


def test_resident_process_exit_right_after_a_call():
    """A process that makes one scalar call (default context, never destroyed) and
    exits at once: the exit handler stops the resident kernel through host memory
    before the runtime tears down; the process exits cleanly."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import tfs_amd.crc as c; "
            "assert c.func_crc(0, bytes(range(256)) * 256) == c.func_crc(0, bytes(range(256)) * 256)" % root)
    for _ in range(3):
        r = subprocess.run([sys.executable, "-c", code], timeout=120, capture_output=True)
        assert r.returncode == 0, r.stderr[-2000:]


def test_resident_contexts_created_and_destroyed_in_turn(oracle):
    """Contexts made and destroyed one after another (page-locked completion memory
    recycled between them): every result of every call is this call's own --
    sequence numbers are process-wide and completion words start zeroed."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(34)
    for c in range(8):
        ctx = crc.Context(0)
        try:
            for it in range(40):
                n = int(rng.integers(1, 6))
                buf, offs, lens = _random_batch(rng, n, maxlen=300000, seed=900 + 40 * c + it)
                seeds = rng.integers(0, 2**32, n).astype(np.uint32)
                assert (ctx.batch(buf, offs, lens, seeds) == _oracle_batch(oracle, buf, offs, lens, seeds)).all(), (c, it)
        finally:
            ctx.close()


def _poisoned_free(ctx, nbytes, word=0x01010101):
    """Allocate nbytes of device memory, fill every 32-bit word with `word` (a
    stale done count / ticket value) and free it, so the next allocation of that
    size is likely to get the same, poisoned, memory back."""
    import tfs_amd.crc as crc
    b = crc.DeviceBuffer(ctx, nbytes)
    b.upload(np.full(nbytes // 4, word, np.uint32))
    ctx.sync()
    p = b.ptr
    b.free()
    return p


def test_resident_state_recycled_from_a_destroyed_context(monkeypatch, oracle):
    """gputests.log:67 of round 2 (a stale done count in a recycled allocation
    made the resident kernel wait for a unit never posted), made deterministic:
    a context runs resident batches (its workgroups' done counts become nonzero)
    and is destroyed; a block of the resident state's size is allocated, filled
    with garbage and freed; a new context's first batch must complete through
    exactly one resident launch -- whether or not it got that memory back."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(35)
    a = _ctx(monkeypatch, TFS_CRC_RESIDENT=1)
    try:
        for it in range(20):
            buf, offs, lens = _random_batch(rng, 7, seed=1200 + it)
            seeds = rng.integers(0, 2**32, 7).astype(np.uint32)
            assert (a.batch(buf, offs, lens, seeds) == _oracle_batch(oracle, buf, offs, lens, seeds)).all()
        st = a.debug_state()
        assert st["res_state"] and st["res_state_bytes"] > 0
        nbytes = st["res_state_bytes"]
    finally:
        a.close()
    for trial in range(3):
        tmp = crc.Context(0)
        garbage = _poisoned_free(tmp, nbytes)
        tmp.close()
        b = _ctx(monkeypatch, TFS_CRC_RESIDENT=1)
        try:
            buf, offs, lens = _random_batch(rng, 5, seed=1300 + trial)
            seeds = rng.integers(0, 2**32, 5).astype(np.uint32)
            t0 = time.perf_counter()
            got = b.batch(buf, offs, lens, seeds)
            dt = time.perf_counter() - t0
            assert (got == _oracle_batch(oracle, buf, offs, lens, seeds)).all(), trial
            launches, files = b.resident_stats()
            assert (launches, files) == (1, 5), (trial, launches, files)
            assert dt < 1.0, dt
            print("trial %d: recycled poisoned block %s" % (trial, b.debug_state()["res_state"] == garbage))
        finally:
            b.close()


def test_resident_poisoned_state_fails_in_bounded_time(monkeypatch, oracle):
    """A batch that can never complete (every workgroup's done count poisoned
    past the ring's published units) returns TFS_CRC_EXIT_DEVICE_ERROR within a
    bounded time instead of hanging, and the context keeps working (it stops
    using the ring and launches)."""
    import tfs_amd.crc as crc
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1, TFS_CRC_RESIDENT_IDLE_US=20)
    try:
        rng = np.random.default_rng(36)
        buf, offs, lens = _random_batch(rng, 3, seed=1400)
        seeds = rng.integers(0, 2**32, 3).astype(np.uint32)
        exp = _oracle_batch(oracle, buf, offs, lens, seeds)
        assert (ctx.batch(buf, offs, lens, seeds) == exp).all()
        time.sleep(0.01)  # past the idle exit: the kernel is gone, its lines are the host's to write
        ctx.debug_poison_resident(1 << 20)
        t0 = time.perf_counter()
        with pytest.raises(crc.TfsCrcError) as e:
            ctx.batch(buf, offs, lens, seeds)
        dt = time.perf_counter() - t0
        assert e.value.code == crc.TFS_CRC_EXIT_DEVICE_ERROR
        assert "no progress" in str(e.value)
        assert dt < 60, dt
        print("poisoned batch failed after %.2f s" % dt)
        assert (ctx.batch(buf, offs, lens, seeds) == exp).all()  # launched from now on
    finally:
        ctx.close()


def test_sched_slots_recycled_from_a_destroyed_context(oracle):
    """The scheduler slots of a new context come zeroed whatever the recycled
    memory held: a garbage-filled block of their size is freed just before the
    context is made, then a dynamic-ticket launch (>= 16 files per wave) and a
    latency-form launch must both be oracle-exact."""
    import tfs_amd.crc as crc
    probe = crc.Context(0)
    nbytes = probe.debug_state()["sched_bytes"]
    probe.close()
    rng = np.random.default_rng(37)
    n = 70000
    lens = rng.integers(0, 200, n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64))
    buf = synth_bytes(1500, int(offs[-1] + lens[-1]) + 64)
    seeds = rng.integers(0, 2**32, n).astype(np.uint32)
    exp = _oracle_batch(oracle, buf, offs, lens, seeds)
    for trial in range(3):
        tmp = crc.Context(0)
        _poisoned_free(tmp, nbytes, word=0x00FFFFFF)
        tmp.close()
        ctx = crc.Context(0)
        try:
            assert (ctx.batch(buf, offs, lens, seeds) == exp).all(), trial
            assert (ctx.batch(buf, offs[:9], lens[:9], seeds[:9]) == exp[:9]).all(), trial
        finally:
            ctx.close()


def test_closes_beside_throughput_launches(oracle):
    """The dataserver's mix on one GPU (data_management.cpp:173-236 beside
    dataservice.cpp:2915-2918 -> task.cpp:713-836): 8 threads closing 64 KiB
    writes through CloseBatcher and the resident kernel, while the same context
    runs verify and compaction launches of 65,536 records (the chunked-ticket
    path).  Both sides' results are checked: every close succeeds, every verdict
    is 1, block 0's compaction equals the oracle's real_compact.  While closes
    flow, throughput launches leave the resident kernel's CUs free (grid 256 - 16);
    with the reserve off, or once the closes have stopped, they take every CU."""
    import tfs_amd.crc as crc
    import tfs_amd.dataserver as ds
    from test_gpu_parity import _oracle_compact
    ctx = crc.Context(0)
    try:
        nblocks, per, rec = 64, 1024, 65536 + 36
        n = nblocks * per
        total = n * rec
        img = crc.DeviceBuffer(ctx, total + 4096)
        ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0xBEEF, 0)
        roff = np.arange(n, dtype=np.uint64) * rec
        desc = np.zeros(n, crc.DESC_DTYPE)
        desc["offset"], desc["len"] = roff + 36, 65536
        d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
        d_crc = crc.DeviceBuffer(ctx, 4 * n)
        ctx.batch_device(d_desc, n, img, d_crc)
        d_roff = crc.DeviceBuffer(ctx, roff.nbytes).upload(roff)
        d_len = crc.DeviceBuffer(ctx, 4 * n).upload(np.full(n, 65536, np.uint32))
        ctx.write_headers_device(img, d_roff, d_len, d_crc, 1, n)
        ctx.sync()
        desc["aux"] = d_crc.download(np.uint32)
        d_v = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
        live = np.arange(0, per, 3)
        nl = live.size
        jobs = np.zeros(nblocks * nl, crc.COMPACT_JOB_DTYPE)
        bidx = np.repeat(np.arange(nblocks, dtype=np.uint64), nl)
        loc = np.tile(np.arange(nl, dtype=np.uint64) * rec, nblocks)
        jobs["src_offset"] = bidx * (per * rec) + np.tile(live.astype(np.uint64) * rec, nblocks)
        jobs["dest_offset"] = bidx * (nl * rec) + loc
        jobs["file_id"] = 1 + bidx * per + np.tile(live.astype(np.uint64), nblocks)
        jobs["size"] = rec
        jobs["new_offset"] = loc.astype(np.int32)
        d_j = crc.DeviceBuffer(ctx, jobs.nbytes).upload(jobs)
        d_dst = crc.DeviceBuffer(ctx, jobs.size * rec + 64)
        d_st = crc.DeviceBuffer(ctx, 4 * jobs.size)
        d_ok = crc.DeviceBuffer(ctx, n)
        d_nb = crc.DeviceBuffer(ctx, 4)
        time.sleep(0.1)  # no resident kernel of an earlier test alive or posted within 50 ms
        assert ctx.throughput_grid() == 256
        for reserve in (True, False):
            ctx.set_cu_reserve(reserve)
            cs = ds.CloseStream(ctx, nleases=8)
            time.sleep(0.05)
            grid = ctx.throughput_grid()
            assert grid == (240 if reserve else 256), (reserve, grid)
            d_nb.zero()
            for _ in range(4):
                d_ok.zero()
                ctx.verify_device(d_v, n, img, None, d_ok, d_nb)
                ctx.compact_jobs_device(img, total, d_j, int(jobs.size), d_dst, None, d_st, d_nb)
            ctx.sync()
            rc, count, lat = cs.stop()
            assert rc == 0 and count > 0, (rc, count)
            assert int(d_nb.download(np.uint32)[0]) == 0
            assert (d_ok.download(np.uint8, n) == 1).all() and (d_st.download(np.int32, jobs.size) == 0).all()
            print("reserve %s: %d closes, p50 %.1f us, p99 %.1f us" % (reserve, count, np.percentile(lat, 50),
                                                                      np.percentile(lat, 99)))
        ctx.set_cu_reserve(True)
        host = img.download(np.uint8, per * rec)
        m = np.zeros(per, crc.META_DTYPE)
        m["file_id"], m["offset"], m["size"] = 1 + np.arange(per), np.arange(per) * rec, rec
        fl = np.where(np.arange(per) % 3 == 0, 0, 1).astype(np.int32)
        odest, _, _ = _oracle_compact(oracle, host, m, fl)
        assert (d_dst.download(np.uint8, odest.size) == odest).all()
        time.sleep(0.1)  # the resident kernel idles out and the last post is > 50 ms old
        assert ctx.throughput_grid() == 256
        for b in (img, d_desc, d_crc, d_roff, d_len, d_v, d_j, d_dst, d_st, d_ok, d_nb):
            b.free()
    finally:
        ctx.close()


def _vram_check(ctx, vram):
    """After the context's first resident call: the ring is where it was asked for
    (device memory needs a large-BAR device; skip when there is none)."""
    where = ctx.resident_ring_in_device_memory()
    if vram and where == 0:
        pytest.skip("no large-BAR device: the ring stays in host memory")
    assert where == vram, where


@pytest.mark.parametrize("vram", [0, 1])
def test_lone_calls_fresh_bytes_every_length(monkeypatch, oracle, vram):
    """Round 6 (units polled by tag, tiny bodies read in one load): lone calls
    through the ring with the content changing on every call -- the scalar drop-in
    on pageable memory (every call through the same reused staging buffer, where
    a stale cached line would show) and page-locked batch calls rewritten in place
    -- lengths 0..100 (bodies of up to 80 bytes travel in the ring unit itself,
    the stripe path above), then random up to 8 KiB, seeds random: every CRC
    equals the oracle's, and every call went through the ring."""
    import tfs_amd.crc as crc
    L = crc.lib()
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1, TFS_CRC_RESIDENT_VRAM=vram)
    pin = crc.PinnedBuffer(ctx, 16384)
    try:
        rng = np.random.default_rng(606)
        lens = list(range(0, 101)) + [int(x) for x in rng.integers(1, 8192, 200)]
        assert L.tfs_crc32_bind_thread(ctx.handle) == 0
        try:
            for k, n in enumerate(lens):
                data = synth_bytes(9000 + k, n + 16).tobytes()
                seed = int(rng.integers(0, 2**32))
                off = k % 13
                assert L.tfs_crc32(seed, data[off:off + n], n) == ocrc(oracle, seed, data[off:off + n]), (k, n)
        finally:
            L.tfs_crc32_bind_thread(None)
        for k, n in enumerate(lens):
            pin.array[:n + 32] = synth_bytes(19000 + k, n + 32)   # rewritten in place every call
            off = (k * 7) % 17
            seed = int(rng.integers(0, 2**32))
            got = ctx.batch(pin.array, [off], [n], [seed])[0]
            assert int(got) == ocrc(oracle, seed, pin.array[off:off + n].tobytes()), (k, n)
        _vram_check(ctx, vram)
        st = ctx.stats()
        nz = sum(1 for n in lens if n > 0)
        assert st["resident_files"] == nz + len(lens), st   # the scalar calls of length 0 never reach the GPU
        assert st["lone_calls"] == nz + len(lens), st
    finally:
        pin.free()
        ctx.close()


@pytest.mark.parametrize("vram", [0, 1])
def test_inline_bodies_mixed_batches_from_threads(monkeypatch, oracle, vram):
    """Bodies of at most 80 bytes travel in their ring unit (tfs_crc_device.h
    kResInline): 8 threads of synchronous verifies, each batch mixing inline
    bodies (0..80 bytes) with bodies read over PCIe (81..3000 bytes), rewritten in
    place every call and with one wrong expected CRC per call, the ring's units
    reused many times over (4,096 units): every CRC and verdict is checked."""
    import tfs_amd.crc as crc
    ctx = _ctx(monkeypatch, TFS_CRC_RESIDENT=1, TFS_CRC_RESIDENT_VRAM=vram)
    errors = []
    nthreads, calls = 8, 400
    try:
        pins = [crc.PinnedBuffer(ctx, 8 * 4096 + 64) for _ in range(nthreads)]

        def worker(t):
            try:
                rng = np.random.default_rng(7000 + t)
                pin = pins[t]
                for it in range(calls):
                    n = int(rng.integers(1, 9))
                    small = rng.random(n) < 0.7
                    lens = np.where(small, rng.integers(0, 81, n), rng.integers(81, 3001, n)).astype(np.uint32)
                    offs = np.arange(n, dtype=np.uint64) * 4096 + rng.integers(0, 16, n).astype(np.uint64)
                    pin.array[:] = rng.integers(0, 256, pin.array.size, dtype=np.uint8)
                    exp = _oracle_batch(oracle, pin.array, offs, lens, np.zeros(n, np.uint32))
                    want = exp.copy()
                    flip = it % n
                    want[flip] ^= 1 << (it % 32)
                    c, ok, nbad, rc = ctx.verify(pin.array, offs, lens, want)
                    if not ((c == exp).all() and nbad == 1 and rc == -1010 and int(np.argmin(ok)) == flip):
                        errors.append((t, it, n, lens.tolist()))
                        return
                    seeds = rng.integers(0, 2**32, n).astype(np.uint32)
                    got = ctx.batch(pin.array, offs, lens, seeds)
                    if not (got == _oracle_batch(oracle, pin.array, offs, lens, seeds)).all():
                        errors.append((t, it, "batch", lens.tolist()))
                        return
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        launches, files = ctx.resident_stats()
        where = ctx.resident_ring_in_device_memory()
        for p in pins:
            p.free()
    finally:
        ctx.close()
    assert not errors, errors[:5]
    assert files > 4096, files  # the ring wrapped
    if vram and where == 0:
        pytest.skip("no large-BAR device: the ring stayed in host memory")
    assert where == vram, where
