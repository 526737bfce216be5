"""Time launch-shape variants of the coordinate-wise median kernel (tool only).

    python tools/median_probe.py        # writes gpurun_out/median_probe.json

Headline shape: 128 clients x 25,610,152 fp32.  Also a compute-only run in
which all 128 table entries point at ONE row (102 MB, served from the caches),
which separates the sorting network's cost from HBM streaming.  Variants run
interleaved in one process; medians reported.
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libmedian_probe.so")
sys.path.insert(0, os.path.dirname(HERE))


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "median_probe.hip")
    deps = [src, os.path.join(HERE, "..", "fedml_amd", "csrc", "fedagg.hip")]
    if not os.path.exists(SO) or max(os.path.getmtime(d) for d in deps) > os.path.getmtime(SO):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-gpu-flush-denormals-to-zero", "-fPIC", "-shared", "-o", SO, src], check=True)
    return SO


def main():
    build()
    from fedml_amd import kernels as kn

    lib = ctypes.CDLL(SO)
    lib.median_probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p]
    lib.median_probe_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    summary = {}
    if "--big-only" not in sys.argv:
        summary.update(probe_k128(lib, kn, dev, st))
    probe_big(lib, kn, dev, st, summary)
    print(json.dumps(summary, indent=1))
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(summary, open("gpurun_out/median_probe.json", "w"), indent=1)


def probe_k128(lib, kn, dev, st):
    K, N = 128, 25_610_152
    L = (N + 63) // 64 * 64
    rows = torch.empty((K, L), device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for i in range(K):
        rows[i].normal_(0.0, 0.05, generator=g)
    tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
    same = kn.upload_i64([rows[0].data_ptr()] * K, dev)
    out = torch.empty(N, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    variants = list(range(6))
    res = {lib.median_probe_name(v).decode(): [] for v in variants}
    res_c = {lib.median_probe_name(v).decode(): [] for v in variants}
    for v in variants:  # warm-up
        assert lib.median_probe_launch(v, tab.data_ptr(), N, out.data_ptr(), st) == 0
    torch.cuda.synchronize()
    for _ in range(5):
        for v in variants:
            name = lib.median_probe_name(v).decode()
            for t, dst in ((tab, res), (same, res_c)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    lib.median_probe_launch(v, t.data_ptr(), N, out.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                dst[name].append(e0.elapsed_time(e1) / 3)
    nbytes = (K + 1) * N * 4
    summary = {}
    for name in res:
        ms = statistics.median(res[name])
        summary[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                         "compute_only_ms": round(statistics.median(res_c[name]), 4)}
    del rows, tab, same, out
    torch.cuda.empty_cache()
    return summary


def probe_big(lib, kn, dev, st, summary):
    """More than 128 clients: LDS-tile radix select (v0), lane-group register
    sort with 128 values per lane (v1) and with 64 per lane (v2), interleaved;
    at K = 128 the shipped pruned network (v4) against two lanes of 64 (v3).
    All outputs must agree bit for bit."""
    lib.median_big_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_void_p]
    names = {0: "radix", 1: "lanes128", 2: "lanes64", 3: "lanes64x2", 4: "net128", 5: "shipped_bs128", 6: "shipped_bs64"}
    N2 = 4_000_000
    for K2 in (128, 129, 256, 257, 512, 513, 1024):
        vs = (4, 3) if K2 <= 128 else (1, 2, 5, 6)
        rows = torch.randn((K2, N2), device=dev) * 0.05
        tab = kn.upload_i64([rows[i].data_ptr() for i in range(K2)], dev)
        outs = {v: torch.empty(N2, device=dev) for v in vs}
        ts = {v: [] for v in vs}
        for v in vs:
            assert lib.median_big_probe(v, tab.data_ptr(), K2, N2, outs[v].data_ptr(), st) == 0
        torch.cuda.synchronize()
        ref = outs[vs[0]].view(torch.int32)
        same_bits = all(bool(torch.equal(ref, outs[v].view(torch.int32))) for v in vs[1:])
        for _ in range(5):
            for v in vs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.median_big_probe(v, tab.data_ptr(), K2, N2, outs[v].data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                ts[v].append(e0.elapsed_time(e1))
        for v in vs:
            ms = statistics.median(ts[v])
            summary[f"{names[v]}_K{K2}_N{N2}"] = {"ms": round(ms, 4), "GBps": round((K2 + 1) * N2 * 4 / ms / 1e6, 1)}
        summary[f"K{K2}_variants_agree"] = same_bits
        print(K2, {names[v]: summary[f"{names[v]}_K{K2}_N{N2}"]["ms"] for v in vs}, same_bits, flush=True)
        del rows, tab, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
