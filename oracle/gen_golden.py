#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY: writes tests/golden/crc_vectors.json.

Every expected value is produced by the reference's own Func::crc text
(src/common/func.cpp:426-435 with the table src/common/func.h:128-154), compiled
by oracle/build_ref.sh into oracle/_ref/libref_crc.so, and cross-checked against
the independent identity Func::crc(c, d) == ~zlib.crc32(d, ~c).
Run in the survey/build container only (it needs /root/reference to build the
.so); the committed JSON is what the tests read.

Inputs are either inline hex (small cases) or a splitmix64 stream
(tfs_amd/synth.py: seed, length, byte offset) that tests regenerate.
"""
import ctypes
import json
import os
import random
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from tfs_amd.synth import synth_bytes  # noqa: E402

PACKET_SEED = 0x4E534654  # TFS_PACKET_FLAG_V1, src/common/base_packet.h:348


def load_ref():
    lib = ctypes.CDLL(os.path.join(HERE, "_ref", "libref_crc.so"))
    lib.ref_func_crc.restype = ctypes.c_uint32
    lib.ref_func_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    return lib


def zlib_identity(seed, data):
    return (~zlib.crc32(data, (~seed) & 0xFFFFFFFF)) & 0xFFFFFFFF


def main():
    ref = load_ref()

    def rcrc(seed, data, n=None):
        n = len(data) if n is None else n
        return ref.ref_func_crc(seed, data, n)

    vec = []

    def add(name, seed, data=None, gen=None, n=None, check_zlib=True):
        if gen is not None:
            data = synth_bytes(gen["seed"], gen["len"], gen.get("offset", 0)).tobytes()
        exp = rcrc(seed, data, n)
        if check_zlib and (n is None or n == len(data)):
            z = zlib_identity(seed, data)
            assert z == exp, (name, hex(z), hex(exp))
        e = {"name": name, "seed": seed, "expected": exp}
        if gen is not None:
            e["gen"] = gen
        else:
            e["hex"] = data.hex()
        if n is not None:
            e["len_arg"] = n
        vec.append(e)

    # Known answers.
    add("kat_123456789_seed0", 0, b"123456789")
    add("kat_123456789_seedffffffff", 0xFFFFFFFF, b"123456789")
    add("kat_123456789_packet_seed", PACKET_SEED, b"123456789")
    add("kat_byte_80", 0, b"\x80")
    add("kat_byte_ff", 0, b"\xff")
    add("kat_byte_00", 0, b"\x00")
    add("kat_empty_seed", 0x12345678, b"")
    add("kat_negative_len", 7, b"abcde", n=-5, check_zlib=False)
    add("kat_zero_len_nonempty_buf", 0xDEADBEEF, b"abc", n=0, check_zlib=False)
    vec.append({"name": "kat_64k_zeros", "seed": 0, "fill": 0, "len": 65536,
                "expected": rcrc(0, bytes(65536))})
    vec.append({"name": "kat_64k_ff", "seed": 0, "fill": 255, "len": 65536,
                "expected": rcrc(0, b"\xff" * 65536)})
    # mock dataserver payload {'1', 0 x 31} (src/tools/mock/mock_data_server_instance.cpp:38-55)
    add("kat_mock_ds_32B", 0, b"1" + bytes(31))

    # Table pin: Func::crc(0, {b}) == _crc32tab[b] for every byte value.
    for b in range(256):
        add("table_%03d" % b, 0, bytes([b]))

    rng = random.Random(20261015)
    seeds = [0, PACKET_SEED, 0xFFFFFFFF, 0x9E3779B9]
    lengths = list(range(0, 258)) + [4095, 4096, 4097, 65535, 65536, 65537,
                                     (1 << 20) - 1, 1 << 20, (1 << 20) + 1]
    for n in lengths:
        s = seeds[n % len(seeds)]
        off = rng.randrange(0, 16)
        add("len_%d_seed%08x_off%d" % (n, s, off), s, gen={"seed": 1000 + n, "len": n, "offset": off})
    # random seeds on mid sizes
    for k in range(16):
        n = rng.randrange(8, 9000)
        s = rng.getrandbits(32)
        add("rand_seed_%d_len%d" % (k, n), s, gen={"seed": 5000 + k, "len": n})

    # Continuation: crc(crc(s, A), B) == crc(s, A||B) (data_file.cpp:183-186 chunking).
    cont = []
    for k in range(12):
        n = rng.randrange(16, 300000)
        cut = rng.randrange(0, n + 1)
        s = rng.choice(seeds)
        d = synth_bytes(9000 + k, n).tobytes()
        c1 = rcrc(s, d[:cut])
        c2 = rcrc(c1, d[cut:])
        assert c2 == rcrc(s, d)
        cont.append({"name": "cont_%d" % k, "gen": {"seed": 9000 + k, "len": n}, "cut": cut,
                     "seed": s, "expected_first": c1, "expected": c2})

    # DataFile::get_crc above the 2 MiB tmp-buffer threshold (data_file.cpp:172-187).
    big = []
    for k, n in enumerate([(2 << 20) + 1, (5 << 20) + 12345]):
        d = synth_bytes(777 + k, n).tobytes()
        c = 0
        off = 0
        while off < n:
            r = min(2 << 20, n - off)
            c = rcrc(c, d[off:off + r])
            off += r
        assert c == rcrc(0, d)
        big.append({"name": "datafile_%d" % n, "gen": {"seed": 777 + k, "len": n}, "expected": c})

    out = {
        "_about": "Golden CRC vectors from the reference Func::crc (src/common/func.cpp:426-435, "
                  "table src/common/func.h:128-154) compiled by oracle/build_ref.sh; generated by "
                  "oracle/gen_golden.py; inputs: inline hex, constant fill, or tfs_amd/synth.py splitmix64 streams.",
        "vectors": vec,
        "continuation": cont,
        "datafile_big": big,
    }
    dst = os.path.join(ROOT, "tests", "golden", "crc_vectors.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote %s: %d vectors, %d continuation, %d big" % (dst, len(vec), len(cont), len(big)))


if __name__ == "__main__":
    main()
