"""Time the lane-group median kernel's launch shapes for 128 < K <= 1024
(tool only; tests/test_gpu_defense.py is the parity check).

    python tools/median_lanes_probe.py [out.json]   # default gpurun_out/median_lanes_probe.json

For each K, every shape that fits runs interleaved in one process on the same
4,000,037 fp32 columns (base ~ N(0, 0.05^2) + 0.01 N(0, 1) per client, as in
tools/median_bench.py), 3 warm-up then 7 timed launches each (HIP events on
the launch stream, median reported), and all outputs must agree bit for bit.
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
SO = os.path.join(HERE, "_build", "libmedian_lanes_probe.so")
sys.path.insert(0, os.path.dirname(HERE))
NV = 8
SHAPE = {0: 256, 1: 512, 2: 512, 3: 1024, 4: 256, 5: 512, 6: 512, 7: 1024}


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "median_lanes_probe.hip")
    deps = [src, os.path.join(HERE, "..", "fedml_amd", "csrc", "fedagg.hip")]
    if not os.path.exists(SO) or max(os.path.getmtime(d) for d in deps) > os.path.getmtime(SO):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-gpu-flush-denormals-to-zero", "-fPIC", "-shared", "-o", SO, src], check=True)
    return SO


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/median_lanes_probe.json"
    build()
    from fedml_amd import kernels as kn

    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.lanes_probe_launch.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int64, P, P]
    lib.lanes_probe_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    N = 4_000_037
    L = (N + 63) // 64 * 64
    res = {"N": N, "shapes": {}}
    for K in [int(k) for k in os.environ.get("PROBE_KS", "256,384,512,768,1024").split(",")]:
        rows = torch.empty((K, L), device=dev)
        g = torch.Generator(device=dev).manual_seed(K)
        base = torch.randn(L, generator=g, device=dev) * 0.05
        for i in range(K):
            rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
        del base
        tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
        vs = [v for v in range(NV) if K <= SHAPE[v] <= 4 * K]  # every shape that holds K
        outs = {v: torch.empty(L, device=dev) for v in vs}
        ts = {v: [] for v in vs}
        for rep in range(10):
            for v in vs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.lanes_probe_launch(v, tab.data_ptr(), K, N, outs[v].data_ptr(), st)
                e1.record()
                assert rc == 0, (v, K, rc)
                torch.cuda.synchronize()
                if rep >= 3:
                    ts[v].append(e0.elapsed_time(e1))
        ref = outs[vs[0]][:N].view(torch.int32)
        agree = all(bool(torch.equal(ref, outs[v][:N].view(torch.int32))) for v in vs[1:])
        # spot check against torch's lower median on a slice
        sl = rows[:, :4096].float()
        tref = torch.median(sl, dim=0).values
        ok_torch = bool(torch.equal(tref.view(torch.int32), outs[vs[0]][:4096].view(torch.int32)))
        entry = {}
        for v in vs:
            ms = statistics.median(ts[v])
            entry[lib.lanes_probe_name(v).decode()] = {"ms": round(ms, 4), "TBps": round((K + 1) * N * 4 / ms / 1e9, 3)}
        res["shapes"][f"K{K}"] = {"variants": entry, "agree": agree, "matches_torch_slice": ok_torch}
        print(K, entry, agree, ok_torch, flush=True)
        del rows, tab, outs
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
