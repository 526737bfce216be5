"""Measure the achievable HBM read and copy rates on the GPU box (tool only).

    python tools/hbm_probe.py            # writes gpurun_out/hbm_probe.json

Buffers are 8 GiB (well beyond the 256 MiB Infinity Cache); interleaved
rounds in one process, median reported.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libhbm_probe.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "hbm_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(src) > os.path.getmtime(SO):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO, src],
                       check=True)
    return SO


def main():
    build()
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(SO)
    lib.probe_read_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p]
    lib.probe_copy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_void_p]
    nbytes = 8 << 30
    src = torch.ones(nbytes // 4, device=dev)
    dst = torch.empty(nbytes // 8, device=dev)  # copy: 4 GiB in, 4 GiB out
    out = torch.empty(2048 * 8 * 256, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    n4 = src.numel() // 4
    cases = {}
    for grid in (2048, 4096, 8192):
        for u in (4, 8, 16):
            cases[f"read_g{grid}_u{u}"] = (lambda g=grid, uu=u: lib.probe_read_launch(src.data_ptr(), n4,
                                                                                      out.data_ptr(), g, uu, st),
                                           nbytes)
    for grid in (2048, 8192):
        cases[f"copy_g{grid}"] = (lambda g=grid: lib.probe_copy_launch(src.data_ptr(), dst.data_ptr(),
                                                                       dst.numel() // 4, g, st), 2 * dst.numel() * 4)
    times = {k: [] for k in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k, (fn, _) in cases.items():
        assert fn() == 0
    torch.cuda.synchronize()
    for _ in range(7):
        for k, (fn, _) in cases.items():
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1))
    res = {}
    for k, (fn, b) in cases.items():
        med = statistics.median(times[k])
        res[k] = {"median_ms": round(med, 4), "GBps": round(b / med / 1e6, 1), "frac_8TBps": round(b / med / 8e9, 4)}
        print(f"{k:18s} {med:8.3f} ms {b / med / 1e6:8.1f} GB/s", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/hbm_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
