"""Philox4x32-10 known-answer vectors (Random123 kat_vectors, Salmon et al. SC'11)."""
import numpy as np

import oracle

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = oracle.test_philox(1, *ctr, *key)[0]
        assert tuple(int(v) for v in got) == want


def test_uniform_words_look_uniform():
    w = oracle.test_philox(50000, 0, 1, 2, 3, 42, 0).reshape(-1)
    u = (w >> 8).astype(np.float64) / 2**24
    assert abs(u.mean() - 0.5) < 0.005 and abs(u.var() - 1 / 12) < 0.002
