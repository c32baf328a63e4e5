"""Deterministic synthetic payload bytes shared by tests, golden fixtures and bench.

Word i (8 bytes, little-endian) of a stream with seed s is splitmix64(s + (i+1)*GOLDEN),
a counter-based generator, so the host (numpy, here) and the device (the
`tfs_synth_fill` kernel in csrc/tfs_crc_kernels.hip) produce the same bytes for any
slice without sequential state.  The GPU bench fills HBM with the device kernel and
tests cross-check slices of it against this module.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64_words(seed: int, first_word: int, nwords: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(first_word + 1, first_word + 1 + nwords, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def synth_bytes(seed: int, nbytes: int, offset: int = 0) -> np.ndarray:
    """Bytes [offset, offset+nbytes) of the stream with the given seed (uint8 array)."""
    if nbytes <= 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = offset // 8
    w1 = (offset + nbytes + 7) // 8
    words = splitmix64_words(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    s = offset - w0 * 8
    return b[s:s + nbytes].copy()
