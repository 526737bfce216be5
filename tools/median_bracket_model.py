"""Would a sampled bracket pay for the counting median at config 4's 512
clients?  (CPU model, the round-5 kill check for VERDICT r04 item 3.)

    python tools/median_bracket_model.py [--waves 4096]

The counting kernel (csrc/median.hip, median_pk16_count) finds each column's
lower median by 8 + 8 byte-bisection steps of v_sad_u8 over all K keys; 2,048
of its ~3,600 VALU per wave are those sums.  A bracket from a sample (Floyd-
Rivest) would replace the 8 high-byte steps by 2 verification counts (+ a
few bisection steps inside a window) -- but a wave holds 32 columns (P = 4
lanes per column pair, 2 columns per lane) that step in lockstep, so a step
is saved only when EVERY column of the wave lands inside its bracket; one
miss sends the whole wave through the full search after the failed check.

On the bench's synthetic updates (base ~ N(0, 0.05^2), client = base +
0.01 eps; bench.fill_rows), per column and per wave of 32 columns:
  exact high byte from a 16-key sample     (2 checks instead of 8 steps)
  4-value high-byte window around it        (2 checks + 2 steps)
  16-value window                           (2 checks + 4 steps)
and the expected high-byte steps per wave against the 8 of today; plus the
key range per wave, max - min over its 32 columns (bits), which bounds any
deterministic narrowing.
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np
import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    K, C = 512, 32 * a.waves
    base = (rng.standard_normal(C) * 0.05).astype(np.float32)
    x = base[None, :] + 0.01 * rng.standard_normal((K, C)).astype(np.float32)
    xb = torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    key = np.where((xb & 0x8000) != 0, ~xb, xb ^ 0x8000).astype(np.uint16)  # order keys, as the kernel
    ks = np.sort(key, axis=0)
    hi = (ks[(K - 1) // 2] >> 8).astype(int)
    g = (np.sort(key[::32], axis=0)[7] >> 8).astype(int)  # 16 strided keys' lower median
    res = {"clients": K, "columns": C, "columns_per_wave": 32}
    full = 8
    for name, lo_off, width, steps in [("exact", 0, 1, 2), ("window4", 1, 4, 4), ("window16", 7, 16, 6)]:
        ok = ((hi >= g - lo_off) & (hi < g - lo_off + width)).reshape(-1, 32)
        pw = float(ok.all(axis=1).mean())
        res[name] = {"column_hit": round(float(ok.mean()), 4), "wave_hit": round(pw, 4),
                     "high_byte_steps_if_hit": steps,
                     "expected_steps_per_wave": round(pw * steps + (1 - pw) * (steps + full), 2)}
    bits = np.ceil(np.log2(ks[-1].astype(int) - ks[0].astype(int) + 1)).reshape(-1, 32).max(axis=1)
    res["wave_key_range_bits"] = {"median": float(np.median(bits)), "min": float(bits.min()),
                                  "fraction_le_12": float((bits <= 12).mean())}
    res["today_high_byte_steps"] = full
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
