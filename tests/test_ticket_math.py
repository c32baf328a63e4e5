"""Host restatement of the kernels' work split (tfs_crc_kernels.hip: Tickets<IL>
and FileCursor<IL, W, CF, TS>): every ticket of the eight interleaved groups is
handed out once, and the chunk/single mapping of chunked tickets covers every
file of a launch exactly once -- for the long-launch (chunked) and the
short-launch (one file per ticket) forms."""
import numpy as np
import pytest

K_DYN_MIN_PER_WAVE = 16  # tfs_crc_device.h kDynMinPerWave


def gcount(n, g):  # Tickets<true>::gcount
    return (n - g + 7) >> 3 if n > g else 0


def file_of(g, j):  # Tickets<true>::file_of
    return j * 8 + g


def cursor_geometry(n, cf, ts, waves):  # FileCursor::init
    if cf > 1:
        nA = (n - (n >> ts)) // cf if ts > 0 else (n + cf - 1) // cf
        nt = nA + (n - nA * cf) if ts > 0 else nA
        if nt < K_DYN_MIN_PER_WAVE * waves:
            return 1, n, n
        return cf, nA, nt
    return 1, n, n


def files_of_tickets(t, n, cf, nA):  # FileCursor::take, vectorised over tickets t
    chunk = t[t < nA]
    first = np.repeat(chunk * cf, cf) + np.tile(np.arange(cf), chunk.size)
    first = first[first < n]
    single = nA * cf + (t[t >= nA] - nA)
    return np.concatenate([first, single])


@pytest.mark.parametrize("cf,ts", [(1, 0), (2, 0), (3, 0), (4, 0), (16, 0), (4, 3), (4, 2), (2, 3), (3, 3), (4, 5)])
def test_every_file_exactly_once(cf, ts):
    rng = np.random.default_rng(cf * 31 + ts)
    waves = 4096
    ns = [1, 7, 8, 9, 1023, 65535, 65536 * 4 + 3, 1 << 20, (1 << 20) + 777] + [int(x) for x in rng.integers(1, 3 << 20, 6)]
    for n in ns:
        c, nA, nt = cursor_geometry(n, cf, ts, waves)
        tickets = np.concatenate([file_of(g, np.arange(gcount(nt, g), dtype=np.int64)) for g in range(8)])
        assert np.array_equal(np.sort(tickets), np.arange(nt))
        files = files_of_tickets(tickets, n, c, nA)
        seen = np.bincount(files, minlength=n)
        assert seen.size == n and (seen == 1).all(), (n, cf, ts)
        if c > 1 and ts > 0:  # long launches take chunks; the last n >> ts files come one per ticket
            assert nt - nA == n - nA * cf >= n >> ts


def gcount_w(n, g, w):  # Tickets<true, W>::gcount
    rem, lo = n % (8 * w), g * w
    return (n // (8 * w)) * w + ((min(rem - lo, w)) if rem > lo else 0)


def file_of_w(g, j, w):  # Tickets<true, W>::file_of
    return (j // w) * (8 * w) + g * w + j % w


@pytest.mark.parametrize("w", [2, 4, 8])
def test_interleaved_slots_of_w_tickets(w):
    """W consecutive tickets per group slot (variants 15/16 on files, 56-58 on
    chunks): the eight groups still hand out every ticket exactly once."""
    for n in [1, 5, 8 * w - 1, 8 * w, 8 * w + 1, 65536 + 13, 1 << 18, (1 << 18) + 8 * w * 3 + 5]:
        t = np.concatenate([file_of_w(g, np.arange(gcount_w(n, g, w), dtype=np.int64), w) for g in range(8)])
        assert np.array_equal(np.sort(t), np.arange(n)), (w, n)


def hybrid_files(n, cf, hs, waves):  # FileCursor<..., CF, TS, HS>: static chunks, then chunk tickets
    """Files each wave takes in the HS form (measurement variants 86-93): static
    chunks w, w+W, ... below hbase, then tickets over the remaining chunks."""
    if n < K_DYN_MIN_PER_WAVE * waves:
        return None  # short launches keep the plain cursor
    nc = (n + cf - 1) // cf
    hbase = (nc - (nc >> hs)) // waves * waves
    static_chunks = np.arange(hbase, dtype=np.int64)          # wave w: chunks w, w + W, ... (all of them)
    assert np.array_equal(np.sort(static_chunks % waves), np.repeat(np.arange(waves), hbase // waves))
    nt = nc - hbase
    tickets = np.concatenate([file_of(g, np.arange(gcount(nt, g), dtype=np.int64)) for g in range(8)])
    chunks = np.concatenate([static_chunks, hbase + tickets])
    first = np.repeat(chunks * cf, cf) + np.tile(np.arange(cf), chunks.size)
    return first[first < n], hbase, nt


@pytest.mark.parametrize("cf,hs", [(1, 1), (1, 2), (1, 3), (1, 5), (4, 1), (4, 2), (4, 3)])
def test_hybrid_static_then_tickets_every_file_once(cf, hs):
    waves = 4096
    for n in [65535, 65536, 65536 * 4 + 3, 349184, 1 << 20, (1 << 20) + 777]:
        r = hybrid_files(n, cf, hs, waves)
        if r is None:
            assert n < K_DYN_MIN_PER_WAVE * waves
            continue
        files, hbase, nt = r
        seen = np.bincount(files, minlength=n)
        assert seen.size == n and (seen == 1).all(), (n, cf, hs)
        assert hbase % waves == 0 and nt >= ((n + cf - 1) // cf) >> hs
