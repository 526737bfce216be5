"""A/B Krum's chunk table (tool only): pieces cut from each run's start vs at
absolute multiples of FEDAGG_PAIR_CHUNK, for both pair kernels.

    python tools/krum_chunks_ab.py [--rounds 9]

Config 3 (128 clients x ResNet-50's fp32 row, base ~ N(0, 0.05^2) + 0.01 N(0, 1)
per client as bench.py), the shipped library, tables interleaved (HIP events
on the launch stream).  Prints times, the largest relative difference of the
two distance matrices and whether Krum's ranking is the same.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    import numpy as np
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
    base = torch.randn(g.rows.shape[1], generator=gen, device=dev) * 0.05
    for i in range(K):
        g.rows[i].copy_(base + 0.01 * torch.randn(g.rows.shape[1], generator=gen, device=dev))
    del base
    tabs = {m: dfn.weight_chunks(g, nat.PAIR_CHUNK, dev, absolute=(m == "absolute")) for m in ("run", "absolute")}
    for method in ("gram", "exact"):
        ts = {m: [] for m in tabs}
        outs = {}
        for r in range(a.rounds + 1):
            for m, (chunks, n) in tabs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                outs[m] = dfn.pairdist2_rows(g.d_ptrs, K, chunks, n, dev, method)
                e1.record()
                e1.synchronize()
                if r:
                    ts[m].append(e0.elapsed_time(e1))
        d0, d1 = outs["run"].cpu().numpy(), outs["absolute"].cpu().numpy()
        off = ~np.eye(K, dtype=bool)
        rel = float(np.max(np.abs(d0[off] - d1[off]) / np.abs(d0[off])))
        f = 10  # byzantine_client_num as the fixtures
        rank0 = np.argsort(dfn.krum_scores(d0, f), kind="stable")
        rank1 = np.argsort(dfn.krum_scores(d1, f), kind="stable")
        print(f"{method}: run {statistics.median(ts['run']):.4f} ms, absolute {statistics.median(ts['absolute']):.4f} "
              f"ms, pieces {tabs['run'][1]} / {tabs['absolute'][1]}, max rel diff {rel:.3e}, "
              f"same ranking {bool((rank0 == rank1).all())}, same first 10 {bool((rank0[:10] == rank1[:10]).all())}",
              flush=True)


if __name__ == "__main__":
    main()
