"""Median kernel timings at the shapes VERDICT round 1 asked about (tool only).

    python tools/median_bench.py [out.json]     # default gpurun_out/median_bench.json

fp32 K = 100 vs 128 over 25,610,152 columns (config 3's row), bf16 K = 100 vs
128 over 86,567,656 (config 4's row, packed kernel), fp32 K = 129 / 256 / 512 /
1024 over 4,000,037 columns, and the radix path at K = 1025 / 2048 over 1M.
--sixteen: bf16 / f16 rows above 128 clients (the packed lane-group kernel),
up to config 4's full shape (512 x 86,567,656 bf16, 88.6 GB).
Each shape: 3 warm-up launches, then 10 timed with HIP events on the launch
stream; median reported, with the algorithmic bytes ((K + 1) x N x esize)
over that time.
"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd import defense as dfn  # noqa: E402
from fedml_amd import kernels as kn  # noqa: E402

SHAPES = [
    (torch.float32, 128, 25_610_152), (torch.float32, 100, 25_610_152),
    (torch.bfloat16, 128, 86_567_656), (torch.bfloat16, 100, 86_567_656),
    (torch.float32, 129, 4_000_037), (torch.float32, 256, 4_000_037), (torch.float32, 512, 4_000_037),
    (torch.float32, 1024, 4_000_037), (torch.bfloat16, 512, 4_000_037),
    (torch.float32, 1025, 1_000_003), (torch.float32, 2048, 1_000_003), (torch.float32, 2049, 1_000_003),
    (torch.float32, 4096, 1_000_003), (torch.float32, 4097, 1_000_003),
]


def time_shape(dtype, K, N, dev, reps=10, one_row=False):
    L = (N + 63) // 64 * 64
    rows = torch.empty((K, L), dtype=dtype, device=dev)
    g = torch.Generator(device=dev).manual_seed(K)
    base = torch.randn(L, generator=g, device=dev) * 0.05
    for i in range(K):
        rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
    del base
    # one_row: every table entry points at row 0 (served from the caches):
    # the selection's VALU cost alone
    d_ptrs = kn.upload_i64([rows[0 if one_row else i].data_ptr() for i in range(K)], dev)
    out = torch.empty(L, dtype=dtype, device=dev)
    for _ in range(3):
        dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dfn.median_rows(d_ptrs, K, N, out, aligned=True)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = statistics.median(ts)
    nbytes = (K + 1) * N * rows.element_size()
    del rows, out
    torch.cuda.empty_cache()
    return {"dtype": str(dtype).replace("torch.", ""), "K": K, "N": N, "one_row": one_row, "ms": round(ms, 4),
            "TBps": round(nbytes / (ms * 1e-3) / 1e12, 3), "frac_of_8TBps": round(nbytes / (ms * 1e-3) / 8e12, 4)}


def main():
    dev = torch.device("cuda:0")
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = args[0] if args else "gpurun_out/median_bench.json"
    res = []
    shapes = [(dt, K, N, False) for dt, K, N in SHAPES]
    if "--sixteen" in sys.argv:  # 16-bit rows above 128 clients (packed lane-group kernel), config 4's K = 512
        shapes = [(torch.bfloat16, K, 4_000_037, False) for K in (129, 256, 384, 512, 700, 1024)]
        shapes += [(torch.bfloat16, K, 1_000_003, False) for K in (1025, 2048, 4096)]
        shapes += [(torch.float16, 512, 4_000_037, False), (torch.bfloat16, 512, 86_567_656, False)]
    if "--one-row" in sys.argv:
        shapes += [(torch.float32, 128, 25_610_152, True), (torch.float32, 512, 4_000_037, True),
                   (torch.float32, 256, 4_000_037, True), (torch.float32, 1024, 4_000_037, True)]
    for dt, K, N, one in shapes:
        r = time_shape(dt, K, N, dev, one_row=one)
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
