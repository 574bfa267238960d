"""CPU: the counting identities the small-bucket kernels rely on
(heatmap_amd/csrc/hm_kernels.hip, hm_small_sort / hm_small_emit), restated
in numpy and checked against a direct count of distinct cells per level.

A bucket's keys are 2*lg-bit Morton codes (col bits even, row bits odd); the
level-l cell of a code is code >> 2l.  The reference counts every (zoom, row,
col) cell of every point (heatmap.py:109-112); per bucket that is, per level,
the number of distinct code >> 2l and each one's multiplicity.

  * cells per bucket = sum over sorted elements of the levels they end:
    element e ends the levels below ceil(bitlen(code[e] ^ code[e+1]) / 2),
    the last element every level (the per-element count of hm_small_sort);
  * the coarsest levels from a 4^NC-slot histogram of the top 2*NC bits,
    the next level up by summing 4 consecutive slots (hm_small_emit), give
    the same (cell, count) pairs as a direct count.
"""
import numpy as np
import pytest


def _levels_direct(codes, lg, zmask):
    out = {}
    for l in range(lg):
        if not (zmask >> l) & 1:
            continue
        u, c = np.unique(codes >> (2 * l), return_counts=True)
        out[l] = dict(zip(u.tolist(), c.tolist()))
    return out


def _cells_per_element(codes, zmask):
    """hm_small_sort's total: one count per element of the sorted codes."""
    s = np.sort(codes).astype(np.uint32)
    total = 0
    zall = bin(zmask).count("1")
    for e in range(len(s)):
        if e + 1 == len(s):
            total += zall
            continue
        x = int(s[e] ^ s[e + 1])
        hl = (x.bit_length() + 1) // 2            # (33 - clz(x)) >> 1
        total += bin(zmask & ((1 << hl) - 1)).count("1")
    return total


def _levels_histogram(codes, lg, zmask, nc):
    """hm_small_emit's coarse levels: 4^nc slots of code >> 2lc, then sums of
    4 consecutive slots per level up (slot prefixes are Morton codes)."""
    lc = lg - nc if lg >= nc else 0
    slots = np.zeros(4 ** (lg - lc) if lg >= nc else 4 ** lg, np.int64)
    np.add.at(slots, codes >> (2 * lc), 1)
    out = {}
    for l in range(lc, lg):
        if (zmask >> l) & 1:
            out[l] = {p: int(c) for p, c in enumerate(slots.tolist()) if c}
        slots = slots.reshape(-1, 4).sum(axis=1) if slots.size >= 4 else slots
    return out, lc


@pytest.mark.parametrize("lg", [1, 2, 3, 4, 7])
@pytest.mark.parametrize("nk", [1, 2, 17, 64, 238, 512])
def test_per_element_cell_count(lg, nk):
    rng = np.random.default_rng(lg * 1000 + nk)
    for zmask in (0, 1, (1 << lg) - 1, 0b1010101 & ((1 << lg) - 1), (1 << lg) - 1 - 1):
        # clustered codes (hot spots inside the bucket) and uniform ones
        for codes in (rng.integers(0, 4 ** lg, nk), rng.integers(0, max(1, 4 ** lg // 16), nk)):
            direct = _levels_direct(codes, lg, zmask)
            assert _cells_per_element(codes, zmask) == sum(len(v) for v in direct.values())


@pytest.mark.parametrize("lg", [2, 3, 4, 7])
@pytest.mark.parametrize("nc", [3, 4])
def test_coarse_levels_from_histogram(lg, nc):
    rng = np.random.default_rng(7 * lg + nc)
    zmask = (1 << lg) - 1
    for nk in (1, 33, 129, 500):
        codes = rng.integers(0, 4 ** lg, nk)
        hist, lc = _levels_histogram(codes, lg, zmask, nc)
        direct = _levels_direct(codes, lg, zmask)
        for l in range(lc, lg):
            assert hist[l] == direct[l], (lg, nc, nk, l)
