"""FedAvg with many clients and a small model (cross-device shape): K up to
4096 clients x N elements, where the element axis alone cannot fill the GPU
(the client axis is a sequential, bit-exact chain per element).  Reports the
kernel time and the byte rate per shape.

    python tools/manyclient_probe.py
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import kernels as kn  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    res = {}
    for K, N in ((1000, 62_006), (4096, 62_006), (1000, 7_850), (128, 62_006), (1000, 1_000_000)):
        L = (N + 63) // 64 * 64
        rows = torch.randn((K, L), device=dev) * 0.05
        d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
        w = kn.upload_f32([1.0 / K] * K, dev)
        out = torch.empty(L, device=dev)
        kn.wsum_ptrs(torch.float32, d_ptrs, w, K, N, out, True)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            kn.wsum_ptrs(torch.float32, d_ptrs, w, K, N, out, True)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        res[f"K{K}_N{N}"] = {"ms": round(ms, 4), "GBps": round((K + 1) * N * 4 / ms / 1e6, 1)}
        print(K, N, res[f"K{K}_N{N}"], flush=True)
        del rows, d_ptrs, out
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/manyclient_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
