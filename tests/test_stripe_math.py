"""CPU emulation of the kernel's decomposition (tfs_crc_kernels.hip), lane by
lane, against the oracle: stripes counted back from the last 16-byte boundary,
zero-extended front, masked first dword, seed injected into the first four
message bytes (carried to stripe 1 when A is stripe 0's last dword), per-stripe
shift over 63 foreign runs, final (63-lane)*RUN shift + XOR-reduce, serial tail.
Uses the same GF(2) helpers the host builds the device tables from
(crc_math.h), restated here in Python."""
import random

import pytest

from conftest import ocrc
from tfs_amd.synth import synth_bytes

POLY = 0xEDB88320


def mult(a, b):
    m, p = 1 << 31, 0
    while True:
        if a & m:
            p ^= b
            if (a & (m - 1)) == 0:
                break
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def x2n(n, k):
    p, sq = 1 << 31, 1 << 30
    for _ in range(k):
        sq = mult(sq, sq)
    while n:
        if n & 1:
            p = mult(sq, p)
        n >>= 1
        sq = mult(sq, sq)
    return p


T = [[0] * 256 for _ in range(4)]
for i in range(256):
    c = i
    for _ in range(8):
        c = (c >> 1) ^ POLY if c & 1 else c >> 1
    T[0][i] = c
for k in range(1, 4):
    for b in range(256):
        T[k][b] = (T[k - 1][b] >> 8) ^ T[0][T[k - 1][b] & 0xFF]
_SH = {}


def shift(c, n):
    if n not in _SH:
        _SH[n] = x2n(n, 3)
    return mult(_SH[n], c)


def step4(c, w):
    x = c ^ w
    return T[3][x & 255] ^ T[2][(x >> 8) & 255] ^ T[1][(x >> 16) & 255] ^ T[0][x >> 24]


def step1(c, b):
    return (c >> 8) ^ T[0][(c ^ b) & 255]


def emulate(mem, start, ln, seed, run):
    ld = lambda a: int.from_bytes(mem[a:a + 4], "little")
    if ln < 32:
        c = seed
        for i in range(ln):
            c = step1(c, mem[start + i])
        return c
    S = 64 * run
    end = start + ln
    A, B16 = start & ~3, end & ~15
    E = (B16 + 127) & ~127 if run == 16 else B16   # stripe anchor: whole 128-byte lines
    nvalid = 64 - (E - B16) // run
    s, body = start - A, E - A
    ns = (body + S - 1) // S
    sb0 = E - ns * S
    headmask = (0xFFFFFFFF << (8 * s)) & 0xFFFFFFFF
    slo = (seed << (8 * s)) & 0xFFFFFFFF
    shi = (seed >> (32 - 8 * s)) if s else 0
    tot = 0
    for lane in range(64):
        c, lo = 0, sb0 + lane * run
        inj = shi if (lane == 0 and A + 4 == sb0 + S) else 0
        for i in range(run // 4):
            q = lo + 4 * i
            w = ld(q) if A <= q < B16 else 0
            if q == A:
                w = (w & headmask) ^ slo
            if q == A + 4:
                w ^= shi
            c = step4(c, w)
        for r in range(1, ns):
            c_old = c
            c = shift(c, 63 * run)
            if r == 1:
                c ^= inj
            q = sb0 + r * S + lane * run
            for i in range(run // 4):
                c = step4(c, ld(q + 4 * i))
            if r == ns - 1 and lane >= nvalid:
                c = c_old
        k = 63 - lane - (64 - nvalid) + (0 if lane < nvalid else 64)
        for j in range(6):
            if (k >> j) & 1:
                c = shift(c, run << j)
        tot ^= c
    c, q = tot, B16
    while q + 4 <= end:
        c = step4(c, ld(q))
        q += 4
    while q < end:
        c = step1(c, mem[q])
        q += 1
    return c


def test_slice_tables_match_oracle_table(oracle):
    import numpy as np
    tab = np.zeros(256, np.uint32)
    oracle.oracle_table(tab.ctypes.data)
    assert [int(x) for x in tab] == T[0]


@pytest.mark.parametrize("run", [16, 32])
def test_emulated_decomposition_matches_oracle(oracle, run):
    mem = synth_bytes(99, 12000).tobytes()
    rnd = random.Random(run)
    cases = [(0, 32, 0), (1, 33, 5), (3, 100, 0xDEADBEEF), (2, 1025, 0), (7, 4100, 0x4E534654)]
    cases += [(rnd.randrange(0, 64), rnd.randrange(32, 6000), rnd.getrandbits(32)) for _ in range(40)]
    # the stripe-0 edge: payload starts inside the last dword of stripe 0
    S = 64 * run
    for st in (29, 30, 31):
        for ln in range(S, 3 * S):
            e = st + ln
            E = ((e & ~15) + 127) & ~127 if run == 16 else e & ~15
            if (st & ~3) + 4 == E - ((E - (st & ~3) + S - 1) // S) * S + S:
                cases.append((st, ln, 0xA5A5F00D))
                break
    for st, ln, sd in cases:
        assert emulate(mem, st, ln, sd, run) == ocrc(oracle, sd, mem[st:st + ln]), (run, st, ln, sd)


def test_shift_identity(oracle):
    """crc(A||B) = shift(crc(A), |B|) ^ crc(B) for seed 0; leading zeros are free."""
    d = synth_bytes(5, 3000).tobytes()
    for cut in (0, 1, 17, 1024, 2999, 3000):
        a, b = d[:cut], d[cut:]
        assert shift(ocrc(oracle, 0, a), len(b)) ^ ocrc(oracle, 0, b) == ocrc(oracle, 0, d)
    assert ocrc(oracle, 0, bytes(100) + d) == ocrc(oracle, 0, d)


KSEG = 128 * 1024
KSPLIT = 128 * 1024


def split_units(L, seed):
    """split_plan_kernel's cut of a file of L bytes (tfs_crc_kernels.hip): a
    ragged head with the seed, then whole KSEG segments with seed 0."""
    if L <= KSPLIT:
        return None
    K = (L - 1) // KSEG + 1
    head = L - (K - 1) * KSEG
    return [(0, head, seed)] + [(head + (j - 1) * KSEG, KSEG, 0) for j in range(1, K)]


def shift5_table(nbytes):
    """make_shift_table5: 7 chunks of 5 bits (the fold's seg_shift table)."""
    k = x2n(nbytes, 3)
    return [[0 if (j == 6 and e >= 4) else mult(k, e << (5 * j)) for e in range(32)] for j in range(7)]


def shift5(t, c):
    r = 0
    for j in range(7):
        r ^= t[j][(c >> (5 * j)) & 31]
    return r


@pytest.mark.parametrize("L", [KSPLIT + 1, 2 * KSEG, 2 * KSEG + 1, 3 * KSEG - 1, 5 * KSEG + 4097, 9 * (1 << 20) + 3])
def test_split_fold_equals_whole_file(oracle, L):
    """The split plan + fold restated: every unit's Func::crc
    from the oracle, folded by the 5-bit seg_shift table, equals the whole
    file's Func::crc with its seed."""
    rnd = random.Random(L)
    data = synth_bytes(L, L).tobytes()
    t = shift5_table(KSEG)
    for seed in (0, 0x4E534654, rnd.getrandbits(32)):
        units = split_units(L, seed)
        assert units and sum(u[1] for u in units) == L and units[0][1] >= 1 and units[0][1] <= KSEG
        c = ocrc(oracle, units[0][2], data[:units[0][1]])
        for off, ln, sd in units[1:]:
            assert sd == 0 and ln == KSEG
            c = shift5(t, c) ^ ocrc(oracle, 0, data[off:off + ln])
        assert c == ocrc(oracle, seed, data), (L, hex(seed))


def test_split_threshold():
    assert split_units(KSPLIT, 5) is None and split_units(KSPLIT - 1, 5) is None
    assert len(split_units(KSPLIT + 1, 5)) == 2 and split_units(KSPLIT + 1, 5)[0][1] == 1
    assert len(split_units(3 * KSEG, 5)) == 3 and split_units(3 * KSEG, 5)[0][1] == KSEG


# ---- bodies carried in the resident ring unit (tfs_crc_kernels.hip inline_crc) ----
K_RES_INLINE = 8 + 6 * 12


def pack_unit(body, tag):
    """The 8 16-byte parts of a ring unit as the host writes them (tfs_crc_abi.cpp
    resident_post): bytes 0..7 in part 0's address words, 12 bytes a part from part 2."""
    w = list(int.from_bytes((bytes(body) + bytes(80))[4 * i:4 * i + 4], "little") for i in range(20))
    parts = [[w[0], w[1], len(body), tag], [0, 0, 0, tag]]
    for k in range(6):
        parts.append([w[2 + 3 * k], w[3 + 3 * k], w[4 + 3 * k], tag if 8 + 12 * k < len(body) else 0])
    return parts


def emulate_inline(parts, ln, seed):
    """inline_crc lane by lane: dword j's CRC from register 0, moved 4*(nd-1-j) bytes by
    the bits of m (4, 8 bytes: zero-dword steps; 16, 32, 64: the level tables), XOR-reduced
    over lanes 0..31, then the last ln % 4 bytes serially."""
    nd = ln // 4
    c = seed
    if nd:
        acc = 0
        for j in range(32):
            src = 0 if j < 2 else 2 + (j - 2) // 3
            k = j if j < 2 else (j - 2) % 3
            w = parts[src][k] if src < 8 else 0
            if j == 0:
                w ^= seed
            x = step4(0, w)
            m = nd - 1 - j if j < nd else 0
            if m & 1:
                x = step4(x, 0)
            if m & 2:
                x = step4(step4(x, 0), 0)
            for bit in (2, 3, 4):
                if (m >> bit) & 1:
                    x = shift(x, 16 << (bit - 2))
            acc ^= x if j < nd else 0
        c = acc
    if ln & 3:
        j = nd
        src = 0 if j < 2 else 2 + (j - 2) // 3
        k = j if j < 2 else (j - 2) % 3
        w = parts[src][k]
        for i in range(ln & 3):
            c = step1(c, (w >> (8 * i)) & 255)
    return c


def test_inline_body_decomposition_matches_oracle(oracle):
    rng = random.Random(80)
    for ln in range(0, K_RES_INLINE + 1):
        for _ in range(4):
            body = bytes(rng.randrange(256) for _ in range(ln))
            seed = rng.randrange(1 << 32)
            parts = pack_unit(body, 7)
            # the kernel takes only the parts it needs: the two halves and ceil((ln - 8) / 12) body parts
            need = 2 + (max(ln - 8, 0) + 11) // 12
            assert all(p[3] == 7 for p in parts[:need]) and all(p[3] == 0 for p in parts[need:])
            assert emulate_inline(parts, ln, seed) == ocrc(oracle, seed, body), (ln, seed)
