"""A/B the radix-select median probe (tools/median_rsel_probe.hip) against the
shipped median kernels (tool only; tests/ hold the parity tests).

    python tools/median_rsel_probe.py [out.json]

For each (dtype, K, N): rows as tools/median_bench.py, the shipped kernel and
the probe interleaved (2 warm-up, 7 timed launches each, HIP events on the
launch stream), outputs compared bit for bit over all N columns, plus a run
with NaN / ±inf injected into a few columns.
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
SO = os.path.join(HERE, "_build", "libmedian_rsel_probe.so")
sys.path.insert(0, os.path.dirname(HERE))


def build():
    src = os.path.join(HERE, "median_rsel_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(src) > os.path.getmtime(SO):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-Wno-unused-value", "-o", SO, src], check=True)
    return SO


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/median_rsel_probe.json"
    build()
    from fedml_amd import defense as dfn
    from fedml_amd import kernels as kn

    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.rsel_launch.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int64, P, P]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    cases = [(torch.float32, 512, 4_000_037, 0), (torch.float32, 300, 4_000_037, 0),
             (torch.float32, 257, 1_000_003, 0), (torch.float32, 256, 4_000_037, 1),
             (torch.float32, 200, 1_000_003, 1),
             (torch.bfloat16, 512, 4_000_036, 2), (torch.bfloat16, 300, 4_000_036, 2),
             (torch.float16, 512, 4_000_036, 3), (torch.float16, 400, 1_000_002, 3),
             (torch.float32, 512, 4_000_037, 4), (torch.float32, 300, 4_000_037, 4), (torch.float32, 257, 1_000_003, 4)]
    only = os.environ.get("RSEL_VARIANTS")
    if only:
        cases = [cs for cs in cases if str(cs[3]) in only.split(",")]
    res = []
    for dtype, K, N, var in cases:
        L = (N + 63) // 64 * 64
        rows = torch.empty((K, L), dtype=dtype, device=dev)
        g = torch.Generator(device=dev).manual_seed(K)
        base = torch.randn(L, generator=g, device=dev) * 0.05
        for i in range(K):
            rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
        del base
        tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
        o_ref = torch.empty(L, dtype=dtype, device=dev)
        o_new = torch.empty(L, dtype=dtype, device=dev)

        def ref():
            dfn.median_rows(tab, K, N, o_ref, aligned=True)

        def new():
            rc = lib.rsel_launch(var, tab.data_ptr(), K, N, o_new.data_ptr(), st)
            assert rc == 0, rc

        ts = {"shipped": [], "rsel": []}
        reps = int(os.environ.get("RSEL_REPS", "9"))
        for rep in range(reps):
            for name, fn in (("shipped", ref), ("rsel", new)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                if rep >= min(2, reps - 1):
                    ts[name].append(e0.elapsed_time(e1))
        same = bool(torch.equal(o_ref[:N].view(torch.int32), o_new[:N].view(torch.int32)))
        # specials: NaN / ±inf / huge values in a few columns
        cols = torch.tensor([0, 1, 2, 3, 17, 64, N - 1], device=dev)
        rows[5, cols[0]] = float("nan")
        rows[K - 1, cols[1]] = float("inf")
        rows[:K // 2 + 1, cols[2]] = float("-inf")
        rows[3, cols[3]] = -float("nan")
        rows[7, cols[3]] = float("nan")
        rows[:, cols[4]] = 3.0e38
        rows[: K // 3, cols[5]] = -3.3e38
        rows[K // 2, cols[6]] = float("nan")
        ref()
        new()
        torch.cuda.synchronize()
        same_sp = bool(torch.equal(o_ref[:N].view(torch.int32), o_new[:N].view(torch.int32)))
        tm = torch.median(rows[:, :4096].float(), dim=0).values
        ok_torch = bool(torch.equal(tm.view(torch.int32), o_new[:4096].float().view(torch.int32)))
        nbytes = (K + 1) * N * rows.element_size()
        r = {"dtype": str(dtype).replace("torch.", ""), "K": K, "N": N, "variant": var,
             "same_as_shipped": same, "same_with_specials": same_sp, "equal_torch_slice": ok_torch}
        for name, v in ts.items():
            ms = statistics.median(v)
            r[name + "_ms"] = round(ms, 4)
            r[name + "_TBps"] = round(nbytes / (ms * 1e-3) / 1e12, 3)
        print(json.dumps(r), flush=True)
        res.append(r)
        del rows, o_ref, o_new
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
