"""Run the shipped median kernel on one shape, for profiler passes (tool only).

    python tools/median_one.py --dtype f32 --K 512 --N 4000037 [--one-row] [--reps 3]

Rows as in tools/median_bench.py (base ~ N(0, 0.05^2) + 0.01 N(0, 1) per
client).  --one-row points every table entry at row 0 (served from the
caches): the selection's own cost.  Prints the median launch time (HIP events
on the launch stream).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd import defense as dfn  # noqa: E402
from fedml_amd import kernels as kn  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32", choices=sorted(DT))
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--N", type=int, default=4_000_037)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--one-row", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dtype, K, N = DT[a.dtype], a.K, a.N
    L = (N + 63) // 64 * 64
    rows = torch.empty((K, L), dtype=dtype, device=dev)
    g = torch.Generator(device=dev).manual_seed(K)
    base = torch.randn(L, generator=g, device=dev) * 0.05
    for i in range(K):
        rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
    del base
    d_ptrs = kn.upload_i64([rows[0 if a.one_row else i].data_ptr() for i in range(K)], dev)
    out = torch.empty(L, dtype=dtype, device=dev)
    dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dfn.median_rows(d_ptrs, K, N, out, aligned=True)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    nbytes = (K + 1) * N * rows.element_size()
    print(json.dumps({"dtype": a.dtype, "K": K, "N": N, "one_row": a.one_row, "ms": round(ms, 4),
                      "TBps": round(nbytes / (ms * 1e-3) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
