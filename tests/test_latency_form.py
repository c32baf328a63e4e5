"""The latency form (one workgroup of 16 waves per file, small batches) and the
launch protocol shared by every CRC launch: stream-bound scheduler slots that
each launch leaves zeroed, and the completion flag zero-copy host batches spin
on.  Bit-exact against the oracle everywhere; every output is checked, not only
mismatch counts."""
import numpy as np
import pytest

from conftest import ocrc
from test_gpu_parity import _stripe_edge_cases
from tfs_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture
def wg_ctx(monkeypatch):
    """A context whose every CRC launch takes the latency form (TFS_CRC_VARIANT=20)."""
    import tfs_amd.crc as crc
    monkeypatch.setenv("TFS_CRC_VARIANT", "20")
    ctx = crc.Context(0)
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    yield ctx
    ctx.close()


def _oracle_batch(oracle, buf, offs, lens, seeds):
    import tfs_amd.crc as crc
    d = np.zeros(len(offs), crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, seeds
    exp = np.zeros(len(offs), np.uint32)
    oracle.oracle_crc_batch(d.ctypes.data, len(offs), buf.ctypes.data, exp.ctypes.data)
    return exp


@pytest.mark.parametrize("seed_mode", ["zero", "random"])
def test_wg_all_small_lengths_and_alignments(wg_ctx, oracle, seed_mode):
    rng = np.random.default_rng(21 if seed_mode == "zero" else 22)
    lens = np.array(list(range(0, 700)) + [int(x) for x in rng.integers(700, 40000, 200)], np.uint32)
    gaps = (np.arange(lens.size) % 16 + 1).astype(np.uint64)
    offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1]]).astype(np.uint64))
    buf = synth_bytes(123, int(offs[-1] + lens[-1]) + 64)
    seeds = np.zeros(lens.size, np.uint32) if seed_mode == "zero" else rng.integers(0, 2**32, lens.size).astype(
        np.uint32)
    got = wg_ctx.batch(buf, offs, lens, seeds)
    exp = _oracle_batch(oracle, buf, offs, lens, seeds)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16) for i in bad[:10]]


def test_wg_stripe0_seed_edges_and_large(wg_ctx, oracle):
    """Payloads starting in the last dword of stripe 0 (the seed's high bytes go to
    wave 1's lane 0), and sizes whose last stripes fall in every wave."""
    items = _stripe_edge_cases(16, 48)
    items += [(o, n) for o in (0, 3, 13) for n in (1024 * k + r for k in (15, 16, 17, 31, 32, 33, 64, 65)
                                                   for r in (0, 1, 112, 127, 128, 1000))]
    items += [(5, 65536), (36, 65536), (1, (1 << 20) + 3), (7, 3 * (1 << 20) + 17)]
    buf = synth_bytes(4343, max(o + n for o, n in items) + 64)
    raw = buf.tobytes()
    rng = np.random.default_rng(5)
    seeds = [int(x) for x in rng.integers(0, 2**32, len(items))]
    for lo in range(0, len(items), 200):   # batches <= 256 files: the product routing also takes this form
        part = items[lo:lo + 200]
        got = wg_ctx.batch(buf, [o for o, _ in part], [n for _, n in part], seeds[lo:lo + 200])
        for (o, n), sd, g in zip(part, seeds[lo:lo + 200], got):
            assert int(g) == ocrc(oracle, sd, raw[o:o + n]), (o, n)


def test_product_routing_small_batches(gpu_ctx, oracle):
    """The product context sends batches of <= 256 files to the latency form and
    larger ones to the wave-per-file kernel: same CRCs either way."""
    rng = np.random.default_rng(6)
    for n in (1, 2, 8, 64, 255, 256, 257, 1000):
        lens = rng.integers(0, 70000, n).astype(np.uint32)
        offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 9, n).astype(np.uint64))
        buf = synth_bytes(900 + n, int(offs[-1] + lens[-1]) + 64)
        seeds = rng.integers(0, 2**32, n).astype(np.uint32)
        got = gpu_ctx.batch(buf, offs, lens, seeds)
        assert (got == _oracle_batch(oracle, buf, offs, lens, seeds)).all(), n


def test_zero_copy_completion_flag_many_calls(gpu_ctx, oracle):
    """Hundreds of back-to-back zero-copy verifies from one page-locked buffer whose
    bytes change between calls: each call sees its own bytes and its own verdicts
    (completion flag reached, outputs visible)."""
    import tfs_amd.crc as crc
    n, ln = 8, 4096
    pin = crc.PinnedBuffer(gpu_ctx, n * ln)
    try:
        offs = np.arange(n, dtype=np.uint64) * ln
        lens = np.full(n, ln, np.uint32)
        rng = np.random.default_rng(8)
        for it in range(400):
            pin.array[:] = rng.integers(0, 256, n * ln, dtype=np.uint8)
            exp = _oracle_batch(oracle, pin.array, offs, lens, np.zeros(n, np.uint32))
            expected = exp.copy()
            flip = it % n
            expected[flip] ^= 1 << (it % 32)
            c, ok, nbad, rc = gpu_ctx.verify(pin.array, offs, lens, expected)
            assert (c == exp).all(), it
            assert nbad == 1 and rc == -1010 and ok.tolist() == [0 if i == flip else 1 for i in range(n)], it
    finally:
        pin.free()


def test_scalar_func_crc_repeated(oracle):
    """tfs_crc32 (pageable, staged into page-locked memory, zero-copy launch) many times."""
    import tfs_amd.crc as crc
    rng = np.random.default_rng(9)
    for it in range(200):
        n = int(rng.integers(0, 70000))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert crc.func_crc(s, d) == ocrc(oracle, s, d), it


def _device_set(ctx, oracle, n=5000, seed=77):
    import tfs_amd.crc as crc
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 40000, n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[0], lens[:-1]]).astype(np.uint64) + rng.integers(0, 16, n).astype(np.uint64))
    buf = synth_bytes(seed, int(offs[-1] + lens[-1]) + 64)
    exp = _oracle_batch(oracle, buf, offs, lens, np.zeros(n, np.uint32))
    d = np.zeros(n, crc.DESC_DTYPE)
    d["offset"], d["len"], d["aux"] = offs, lens, exp
    d_img = crc.DeviceBuffer(ctx, buf.size).upload(buf)
    d_desc = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
    return d_img, d_desc, exp


def test_back_to_back_launches_reset_their_tickets(gpu_ctx, oracle):
    """30 wave-per-file launches queued on one stream with no synchronisation in
    between: each finds its ticket counters zeroed by the previous one, so every
    file of every launch is computed (every output checked, every verdict 1)."""
    import tfs_amd.crc as crc
    n = 5000
    d_img, d_desc, exp = _device_set(gpu_ctx, oracle, n)
    outs = [crc.DeviceBuffer(gpu_ctx, 4 * n) for _ in range(30)]
    oks = [crc.DeviceBuffer(gpu_ctx, n) for _ in range(30)]
    for o, k in zip(outs, oks):
        o.zero()
        k.zero()
    gpu_ctx.sync()
    for o, k in zip(outs, oks):
        gpu_ctx.verify_device(d_desc, n, d_img, o, k)
    gpu_ctx.sync()
    for o, k in zip(outs, oks):
        assert (o.download(np.uint32) == exp).all()
        assert (k.download() == 1).all()


def test_concurrent_streams_have_their_own_slots(gpu_ctx, oracle):
    """Launches in flight on two streams at once (and the ctx stream): no shared
    ticket counters, so no file is skipped on any stream."""
    import tfs_amd.crc as crc
    n = 6000
    d_img, d_desc, exp = _device_set(gpu_ctx, oracle, n, seed=78)
    streams = [gpu_ctx.stream_create(), gpu_ctx.stream_create(), None]
    rounds = 10
    outs = {(s, r): crc.DeviceBuffer(gpu_ctx, 4 * n) for s in range(3) for r in range(rounds)}
    oks = {(s, r): crc.DeviceBuffer(gpu_ctx, n) for s in range(3) for r in range(rounds)}
    try:
        for b in list(outs.values()) + list(oks.values()):
            b.zero()
        gpu_ctx.sync()
        for r in range(rounds):
            for s, st in enumerate(streams):
                gpu_ctx.verify_device(d_desc, n, d_img, outs[(s, r)], oks[(s, r)], stream=st)
        for st in streams[:2]:
            gpu_ctx.stream_sync(st)
        gpu_ctx.sync()
        for key in outs:
            assert (outs[key].download(np.uint32) == exp).all(), key
            assert (oks[key].download() == 1).all(), key
    finally:
        for st in streams[:2]:
            gpu_ctx.stream_destroy(st)
