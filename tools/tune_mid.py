"""Tile configurations of the fp32 weighted sum at MID sizes (GPU only).

The per-rank sizes of strong scaling (config 3 at 2-8 ranks: 128 x 3.2-12.8M;
config 5 at 2-8 ranks: 64 x 0.52-2.1M) sit between the small-tensor tiles
(SmallCfg, chosen below 1,024 shipped tiles for configs 1-2) and the
mid/large ones.  This sweeps a few variants over a grid of (K, N) in ONE
process, interleaved, R rounds each, and reports the median per variant and
shape, with every variant checked bit for bit against the shipped kernel.

    python tools/tune_mid.py --rounds 25 > gpurun_out/tune_mid.txt
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import _native as nat  # noqa: E402

VARIANTS = ["shipped", "U4V4nt", "U2V4nt", "U1V4nt", "U8V2nt", "U2V2nt", "U4V4nt_b128", "U2V4nt_b128",
            "U4V4nt_b64", "U16V1nt_b64", "U1V8nt"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=25)
    ap.add_argument("--K", type=int, nargs="*", default=[32, 64, 128])
    ap.add_argument("--blocks", type=int, nargs="*", default=[32, 64, 128, 256, 512, 768, 1023, 1536])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from tools import tuning_lib

    lib = tuning_lib.lib()  # the tuning build: the product library has no variant entries
    names = [lib.fedagg_variant_name(v).decode() for v in range(lib.fedagg_num_variants())]
    idx = {n: i for i, n in enumerate(names)}
    st = nat.stream_handle()
    res = {}
    maxK, maxN = max(a.K), max(a.blocks) * 4096
    rows = torch.empty((maxK, maxN), dtype=torch.float32, device=dev).normal_(0.0, 0.05)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for K in a.K:
        ptrs = torch.tensor([rows[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
        w = torch.full((K,), 1.0 / K, dtype=torch.float32, device=dev)
        for B in a.blocks:
            N = B * 4096
            outs = {v: torch.empty(N, device=dev) for v in VARIANTS}
            times = {v: [] for v in VARIANTS}

            def run(v):
                tuning_lib.check(lib.fedagg_wsum_f32_variant(ptrs.data_ptr(), w.data_ptr(), K, N, outs[v].data_ptr(),
                                                      idx[v], st), v)

            for v in VARIANTS:
                run(v)
            torch.cuda.synchronize()
            for v in VARIANTS:
                assert torch.equal(outs[v].view(torch.int32), outs["shipped"].view(torch.int32)), v
            for _ in range(a.rounds):
                for v in VARIANTS:
                    ev0.record()
                    run(v)
                    ev1.record()
                    ev1.synchronize()
                    times[v].append(ev0.elapsed_time(ev1))
            med = {v: statistics.median(t) for v, t in times.items()}
            best = min(med, key=med.get)
            gbs = {v: (K + 1) * N * 4 / m / 1e6 for v, m in med.items()}
            res[f"K{K}_B{B}"] = {"K": K, "N": N, "median_ms": med, "GBps": gbs, "best": best}
            print(f"K={K:4d} B={B:5d} N={N:9d} best {best:12s} {med[best]:.4f} ms {gbs[best]:7.0f} GB/s | "
                  + " ".join(f"{v}={med[v]:.4f}" for v in VARIANTS), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/tune_mid.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
