#!/usr/bin/env python3
"""oracle/gen_golden_ec.py -- TEST INFRASTRUCTURE ONLY: writes tests/golden/ec_vectors.json.

Expected parity (and decode outputs) come from the reference's own vendored
jerasure/galois (src/dataserver/jerasure.cpp, galois.cpp) compiled by
oracle/build_ref.sh into oracle/_ref/libref_ec.so and driven like ErasureCode
(oracle/ec_ref_driver.cpp).  Inputs are splitmix64 streams (tfs_amd/synth.py)
that the tests regenerate: member i of a case is synth_bytes(seed + i, size).
Each case stores sha256 of every parity member plus its first 64 bytes, and
for each erasure pattern the sha256 of every rebuilt member.
Run in the build container only (needs /root/reference); commit the JSON.
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from tfs_amd.synth import synth_bytes  # noqa: E402

CASES = [
    # (k, m, size, seed, erasure patterns)
    (5, 3, 8192, 100, [[0, 0, 0, 0, 1, 0, 1, 1], [1, 1, 0, 0, 0, 0, 0, 1], [0, 0, 0, 1, 1, 1, 0, 0]]),
    (4, 2, 4096, 200, [[1, 0, 0, 0, 0, 1], [0, 1, 1, 0, 0, 0], [0, 0, 0, 0, 1, 1]]),
    (2, 1, 1024, 300, [[1, 0, 0], [0, 0, 1]]),
    (8, 4, 2048, 400, [[1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1],
                       [0, 1, 0, 1, 0, 0, 0, 0, 0, 1, 0, 1]]),
    (10, 2, 3072, 500, [[0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 0], [-1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1]]),
    (1, 1, 1024, 600, [[1, 0], [0, 1]]),
    (3, 9, 1024, 700, [[1, 1, 1, 0, 0, 0, 0, 0, 0, 1, 1, 1]]),
]


def members(k, m, size, seed):
    return [ctypes.create_string_buffer(synth_bytes(seed + i, size).tobytes() if i < k else bytes(size), size)
            for i in range(k + m)]


def main():
    ref = ctypes.CDLL(os.path.join(HERE, "_ref", "libref_ec.so"))
    ref.ref_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    ref.ref_ec_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    out = []
    for k, m, size, seed, patterns in CASES:
        bufs = members(k, m, size, seed)
        ptrs = (ctypes.c_char_p * (k + m))(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs])
        assert ref.ref_ec_encode(k, m, ptrs, size) == 0
        coded = [bytes(b.raw) for b in bufs]
        case = {"k": k, "m": m, "size": size, "seed": seed,
                "parity_sha256": [hashlib.sha256(coded[k + i]).hexdigest() for i in range(m)],
                "parity_head_hex": [coded[k + i][:64].hex() for i in range(m)], "decode": []}
        for er in patterns:
            bufs2 = [ctypes.create_string_buffer(coded[i] if er[i] == 0 else bytes(size), size) for i in range(k + m)]
            ptrs2 = (ctypes.c_char_p * (k + m))(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs2])
            e = (ctypes.c_int * (k + m))(*er)
            rc = ref.ref_ec_decode(k, m, e, ptrs2, size)
            rebuilt = {str(i): hashlib.sha256(bytes(bufs2[i].raw)).hexdigest() for i in range(k + m) if er[i] != 0}
            case["decode"].append({"erased": er, "rc": rc, "rebuilt_sha256": rebuilt if rc == 0 else {}})
            if rc == 0:  # a correct decode restores the coded members
                for i in range(k + m):
                    if er[i] == 1 or (i < k and er[i] != 0):
                        assert bytes(bufs2[i].raw) == coded[i], (k, m, er, i)
        out.append(case)
    path = os.path.join(ROOT, "tests", "golden", "ec_vectors.json")
    with open(path, "w") as f:
        json.dump({"generator": "oracle/gen_golden_ec.py via oracle/_ref/libref_ec.so "
                                "(reference src/dataserver/jerasure.cpp + galois.cpp)", "cases": out}, f, indent=1)
    print("wrote", path, len(out), "cases")


if __name__ == "__main__":
    main()
