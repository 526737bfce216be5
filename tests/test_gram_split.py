"""The arithmetic behind the split-bf16 centred Gram (csrc/robust.hip,
pairgram_split_kernel / pairgram_split8_kernel), restated in numpy:

- the three-way split of an fp32 value into bf16 parts, h = bf16(c),
  m = bf16(c - h), l = bf16(c - h - m) (each rounded to nearest even, as
  v_cvt_pk_bf16_f32 does), is EXACT: c == h + m + l for every finite fp32
  value whose parts stay normal;
- the six products the kernel keeps (hh, hm, mh, mm, hl, lh) differ from the
  exact product c_i c_j by at most 2^-23 |c_i| |c_j| (|m| <= 2^-8 |c|,
  |l| <= 2^-8 |m|: the dropped m l + l m + l l), the order of the fp32
  rounding of each product on the f32 MFMA (2^-24).
"""
from __future__ import annotations

import numpy as np


def _bf16_rne(x: np.ndarray) -> np.ndarray:
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32)


def _split(c: np.ndarray):
    c = c.astype(np.float32)
    h = _bf16_rne(c)
    r = (c - h).astype(np.float32)  # exact in fp32
    m = _bf16_rne(r)
    l32 = (r - m).astype(np.float32)  # exact in fp32
    l_ = _bf16_rne(l32)
    return h, m, l_, l32


def test_three_way_bf16_split_is_exact():
    rng = np.random.default_rng(0)
    # centred model updates: every magnitude from 1e-30 to 1e30, both signs
    c = (rng.standard_normal(200_000) * 10.0 ** rng.uniform(-30, 30, 200_000)).astype(np.float32)
    c = np.concatenate([c, np.float32([0.0, -0.0, 1.0, -1.0, 3.0e38, -3.0e38, 1.17549435e-38])])
    h, m, l_, l32 = _split(c)
    assert (l_ == l32).all(), "the third part must already be a bf16 value"
    s = h.astype(np.float64) + m.astype(np.float64) + l_.astype(np.float64)
    np.testing.assert_array_equal(s, c.astype(np.float64))
    # each part has at most 8 significant bits (a bf16): the low 16 bits are zero
    for part in (h, m, l_):
        assert (part.view(np.uint32) & 0xFFFF == 0).all()


def test_six_products_bound():
    rng = np.random.default_rng(1)
    a = (rng.standard_normal(100_000) * 10.0 ** rng.uniform(-6, 2, 100_000)).astype(np.float32)
    b = (rng.standard_normal(100_000) * 10.0 ** rng.uniform(-6, 2, 100_000)).astype(np.float32)
    ha, ma, la, _ = _split(a)
    hb, mb, lb, _ = _split(b)
    f = np.float64
    kept = (f(ha) * f(hb) + f(ha) * f(mb) + f(ma) * f(hb) + f(ma) * f(mb) + f(ha) * f(lb) + f(la) * f(hb))
    exact = f(a) * f(b)
    assert (np.abs(kept - exact) <= 2.0 ** -23 * np.abs(exact)).all()
    # and the dropped terms are what makes the difference
    dropped = f(ma) * f(lb) + f(la) * f(mb) + f(la) * f(lb)
    np.testing.assert_allclose(kept + dropped, exact, rtol=0, atol=1e-300)


def test_block_schedule_covers_the_triangle_once():
    """pairgram_split8_kernel's 2 x 2 group-block schedule at 8 groups
    (csrc/robust.hip, kBlk8 / kBlk8Tile): every tile (a <= b) of the 8 x 8
    group triangle exactly once, 9 tiles per SIMD (waves s and s + 4), and the
    slot table agrees with the blocks' order (A0B0, A0B1, A1B0 unless diagonal,
    A1B1)."""
    import os
    import re

    src = open(os.path.join(os.path.dirname(__file__), "..", "fedml_amd", "csrc", "robust.hip")).read()

    def table(name):
        body = src[src.index(name):]
        body = body[body.index("{"):body.index("};") + 1]
        body = re.sub(r"//[^\n]*", "", body)  # comments
        return [int(x) for x in re.findall(r"-?\d+", body)]

    blk = table("constexpr int kBlk8[8][2][5]")
    tiles = table("kBlk8Tile[8][5][2]")
    assert len(blk) == 80 and len(tiles) == 80
    seen = []
    for w in range(8):
        slots = []
        for k in range(2):
            a0, a1, b0, b1, diag = blk[w * 10 + k * 5: w * 10 + k * 5 + 5]
            if a0 < 0:
                continue
            slots.append((a0, b0))
            if b1 >= 0:
                slots.append((a0, b1))
            if not diag:
                slots.append((a1, b0))
            if b1 >= 0:
                slots.append((a1, b1))
        want = [(tiles[w * 10 + 2 * j], tiles[w * 10 + 2 * j + 1]) for j in range(5)]
        want = [t for t in want if t[0] >= 0]
        assert slots == want, w
        seen += slots
    assert sorted(seen) == [(a, b) for a in range(8) for b in range(a, 8)]
    per_simd = [sum(1 for w in (s, s + 4) for j in range(5) if tiles[w * 10 + 2 * j] >= 0) for s in range(4)]
    assert per_simd == [9, 9, 9, 9]
