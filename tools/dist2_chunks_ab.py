"""A/B dist2's chunk table: pieces cut from each run's start vs at absolute
multiples of the chunk (tool only; tests/ hold the parity tests).

    python tools/dist2_chunks_ab.py [--rounds 15] [--only run|absolute]

Config 3 (128 clients x ResNet-50's fp32 row, rows as tools/robust_variants.py),
the shipped library, the two tables interleaved (HIP events on the launch
stream); the two results must agree to fp64 rounding.  --only times one table
(for a FETCH_SIZE pass).
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--only", choices=["run", "absolute"], default=None)
    a = ap.parse_args()
    import torch

    from fedml_amd import _native as nat
    from fedml_amd import defense as dfn
    from fedml_amd import shapes
    from fedml_amd.bucket import ClientBucket

    dev = torch.device("cuda:0")
    K = 128
    b = ClientBucket(shapes.resnet50(), K, dev)
    g = b.groups[torch.float32]
    gen = torch.Generator(device=dev).manual_seed(0)
    g.rows.normal_(0.0, 0.05, generator=gen)
    ref = g.rows[K - 1].clone()
    tabs = {}
    for mode in ("run", "absolute"):
        if a.only in (None, mode):
            tabs[mode] = dfn.weight_chunks(g, nat.DIST_CHUNK, dev, absolute=(mode == "absolute"))
    n_w = sum(n for k, n in zip(g.keys, g.numels) if dfn.is_weight_param(k))
    outs, ts = {}, {m: [] for m in tabs}
    for r in range(a.rounds + 1):
        for mode, (chunks, n_chunks) in tabs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            d = dfn.dist2_rows(g.d_ptrs, K, ref, chunks, n_chunks, dev)
            e1.record()
            e1.synchronize()
            outs[mode] = d
            if r:
                ts[mode].append(e0.elapsed_time(e1))
    if len(outs) == 2:
        assert torch.allclose(outs["run"], outs["absolute"], rtol=1e-13, atol=0), "tables disagree"
    alg = (K + 1) * n_w * 4
    for mode, t in ts.items():
        m = statistics.median(t)
        print(f"dist2 {mode:9s} pieces {tabs[mode][1]:6d}  median {m:.4f} ms  {alg / m / 1e6:7.1f} GB/s "
              f"({alg / m / 1e6 / 8000:.3f})  alg bytes {alg}", flush=True)


if __name__ == "__main__":
    main()
