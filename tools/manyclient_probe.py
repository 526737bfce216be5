"""FedAvg with many clients and a small model (cross-device shape): K up to
4096 clients x N elements, where the element axis alone cannot fill the GPU
(the client axis is a sequential, bit-exact chain per element).  Reports the
kernel time and the byte rate per shape.

    python tools/manyclient_probe.py [--dtype bf16] [--out name]
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
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"])
    ap.add_argument("--acc", default="reference", choices=["reference", "fp32"])
    ap.add_argument("--out", default="manyclient_probe")
    a = ap.parse_args()
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    acc = kn.ACC_REFERENCE if a.acc == "reference" else kn.ACC_FP32
    esz = torch.empty((), dtype=dt).element_size()
    dev = torch.device("cuda:0")
    res = {}
    for K, N in ((1000, 62_006), (4096, 62_006), (1000, 7_850), (128, 62_006), (1000, 1_000_000)):
        L = (N + 63) // 64 * 64
        rows = (torch.randn((K, L), device=dev) * 0.05).to(dt)
        d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
        w = kn.upload_f32([1.0 / K] * K, dev)
        out = torch.empty(L, device=dev, dtype=dt)
        kn.wsum_ptrs(dt, d_ptrs, w, K, N, out, True, acc)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            kn.wsum_ptrs(dt, d_ptrs, w, K, N, out, True, acc)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        res[f"K{K}_N{N}"] = {"ms": round(ms, 4), "GBps": round((K + 1) * N * esz / ms / 1e6, 1)}
        print(a.dtype, a.acc, K, N, res[f"K{K}_N{N}"], flush=True)
        del rows, d_ptrs, out
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open(f"gpurun_out/{a.out}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
