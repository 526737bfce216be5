"""The counting median's per-byte search (csrc/median.hip, sad_bisect), and
the Fibonacci search over the same convex sum that was measured against it
in round 4 (13 sums instead of 16, but more VALU per wave in total:
3,885 vs 3,619, equal time; profiles/r04/i/), restated step for step in
Python and checked exhaustively against the sorted order statistic (CPU).
The GPU kernels themselves are pinned by tests/test_gpu_defense.py against
the reference's fixtures."""
from __future__ import annotations

import numpy as np
import pytest

FIB = [1, 1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144, 233, 377]


def _sums(counts: np.ndarray):
    """S(p) = sum |byte - p| for p in [0, 255] from a byte histogram, and the
    extension past 255 the kernel uses (S(255) + (p - 255) n)."""
    vals = np.arange(256)
    n = int(counts.sum())
    table = np.array([int((np.abs(vals - p) * counts).sum()) for p in range(256)])

    def S(p):
        return int(table[min(p, 255)]) + max(p - 255, 0) * n
    return S


def fibonacci(S):
    """The Fibonacci variant for one column: 13 probes, the interval padded to 377."""
    a, x1, x2 = 0, FIB[11] - 1, FIB[12] - 1
    f1, f2 = S(x1), S(x2)
    probes = 2
    for k in range(13, 3, -1):
        c = f1 <= f2
        p = a + FIB[k - 3] - 1 if c else x1 + FIB[k - 2]
        if c:
            x2, f2 = x1, f1
        else:
            a, x1, f1 = x1 + 1, x2, f2
        g = S(p)
        probes += 1
        if c:
            x1, f1 = p, g
        else:
            x2, f2 = p, g
    assert x1 == a and x2 == a + 1
    g = S(a + 2)
    probes += 1
    return (a if f1 <= f2 else (a + 1 if f2 <= g else a + 2)), probes


def bisect(S, n):
    """sad_bisect: the smallest v with #(byte <= v) >= n / 2, two sums per step."""
    v = 0
    for bit in range(7, -1, -1):
        p = v + (1 << bit) - 1
        if S(p + 1) - S(p) < 0:
            v += 1 << bit
    return v


def _cases():
    rng = np.random.default_rng(0)
    for n in (256, 512, 1024):
        yield rng.integers(0, 256, n)
        yield rng.integers(100, 140, n)
        yield rng.choice([0, 255], n)
        yield rng.choice([7, 8], n)
        yield rng.integers(250, 256, n)
        yield rng.integers(0, 6, n)
        yield np.full(n, 0)
        yield np.full(n, 255)
        yield np.full(n, 128)
        # half exactly at one value, half above / below: the median sits on a plateau edge
        yield np.concatenate([np.full(n // 2, 37), np.full(n // 2, 200)])
        yield np.concatenate([np.full(n // 2 - 1, 37), np.full(n // 2 + 1, 200)])
        yield np.concatenate([np.full(n // 2 + 1, 37), np.full(n // 2 - 1, 200)])
        for _ in range(300):
            lo = int(rng.integers(0, 256))
            hi = int(rng.integers(lo, 256)) + 1
            yield rng.integers(lo, hi, n)


@pytest.mark.parametrize("search", ["fibonacci", "bisect"])
def test_byte_search_finds_the_lower_median(search):
    for keys in _cases():
        n = keys.size
        counts = np.bincount(keys, minlength=256)
        S = _sums(counts)
        want = int(np.sort(keys)[n // 2 - 1])  # the lower median: KMAX/2 keys at or below it
        if search == "fibonacci":
            got, probes = fibonacci(S)
            assert probes == 13
        else:
            got = bisect(S, n)
        assert got == want, (search, n, want, got)
