"""The packed 16-bit median above 128 clients, as shipped and beside its
register forms (tool only; tests/test_gpu_defense.py is the parity check).

    python tools/median_slice_probe.py [out.json]   # default gpurun_out/median_slice_probe.json

Variants (median_slice_probe.hip: slice_probe_name): 1 the product dispatch
(LDS-DMA streamed bit-plane select), 2 the register form of the bit-plane
select, 3 the sorting networks, 4 the column kernel at 32 words per lane in
8-wave blocks.  All run on the same rows and must agree bit
for bit with the first variant listed:
  - edge shapes first (K = 129 .. 1024 incl. padding, odd N for the tail
    launch, f16 and bf16, NaN / +-inf / +-0 / denormal columns, all-equal and
    two-valued columns), each also against torch.median's value;
  - then the timed shapes, interleaved in one process: 3 warm-ups, then
    PROBE_REPS launches of each (HIP events on the launch stream, median),
    bf16 K = 512 over config 4's 86,567,656 columns (88.8 GB) last;
    one_row: every table entry points at row 0 (the selection's cost alone).
PROBE_VARIANTS picks variants (default 1,2); PROBE_QUICK=1 skips the edge
shapes and keeps K = 512 over 8M columns, =2 adds config 4's full shape.
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
SO = os.path.join(HERE, "_build", "libmedian_slice_probe.so")
sys.path.insert(0, os.path.dirname(HERE))


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "median_slice_probe.hip")
    deps = [src, os.path.join(HERE, "..", "fedml_amd", "csrc", "median.hip")]
    if not os.path.exists(SO) or max(os.path.getmtime(d) for d in deps) > os.path.getmtime(SO):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-gpu-flush-denormals-to-zero", "-fPIC", "-shared", "-o", SO, src], check=True)
    return SO


def rows_for(K, N, dtype, dev, seed, specials=False):
    L = (N + 63) // 64 * 64
    rows = torch.empty((K, L), dtype=dtype, device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    base = torch.randn(L, generator=g, device=dev) * 0.05
    for i in range(K):
        rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
    if specials:
        n = min(N, 4096)
        col = torch.arange(n, device=dev)
        kind = col % 8
        for i in range(K):
            r = rows[i, :n]
            r[kind == 1] = float("nan") if i == (7 * int(seed)) % K else r[kind == 1]
            r[kind == 2] = float("inf") if i % 3 == 0 else -float("inf") if i % 3 == 1 else 0.0
            r[kind == 3] = 0.0 if i % 2 else -0.0
            r[kind == 4] = 1.5
            r[kind == 5] = 1e-40 if i % 2 else -1e-40
            r[kind == 6] = float(i % 2)
            r[kind == 7] = float(-(i % 5))
    return rows


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/median_slice_probe.json"
    build()
    from fedml_amd import kernels as kn

    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.slice_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int64, P, P]
    lib.slice_probe_name.restype = ctypes.c_char_p
    variants = [int(v) for v in os.environ.get("PROBE_VARIANTS", "1,2").split(",")]
    names = {v: lib.slice_probe_name(v).decode() for v in variants}
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    res = {"edge": [], "timed": []}

    def run(sel, f16, tab, K, N, out):
        rc = lib.slice_probe_launch(sel, f16, tab.data_ptr(), K, N, out.data_ptr(), st)
        assert rc == 0, rc

    # edge shapes: bit-exact agreement, and torch.median's value on every column (sign of a zero aside)
    for dtype in (() if os.environ.get("PROBE_QUICK") else (torch.bfloat16, torch.float16)):
        f16 = int(dtype == torch.float16)
        for K, N in (((1, 999), (2, 1000), (5, 1001), (31, 3000), (33, 3001), (64, 2048), (65, 2049), (100, 4097),
                      (127, 2049), (128, 4098)) if os.environ.get("PROBE_SMALLK") else ()) + ((129, 5001), (200, 4096), (256, 4097), (300, 3333), (511, 4096), (512, 4099), (513, 2049),
                     (700, 4097), (1024, 4096)):
            rows = rows_for(K, N, dtype, dev, seed=K + 17 * f16, specials=True)
            tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
            outs = {v: torch.full((N,), 7, dtype=dtype, device=dev) for v in variants}
            for v in variants:
                run(v, f16, tab, K, N, outs[v])
            torch.cuda.synchronize()
            b1 = outs[variants[0]].view(torch.int16)
            diffs = {names[v]: int((b1 != outs[v].view(torch.int16)).sum()) for v in variants[1:]}
            ref = rows[:, :N].float().median(dim=0).values.to(dtype)
            o2 = outs[variants[0]]
            same_val = (ref.view(torch.int16) == o2.view(torch.int16)) | ((ref == 0) & (o2 == 0)) | (
                ref.isnan() & o2.isnan())
            r = {"dtype": str(dtype)[6:], "K": K, "N": N, "diff_vs_first": diffs,
                 "diff_vs_torch_value": int((~same_val).sum())}
            print(json.dumps(r), flush=True)
            res["edge"].append(r)
            assert not any(diffs.values()), r
            del rows, tab
    torch.cuda.empty_cache()

    reps = int(os.environ.get("PROBE_REPS", "10"))
    shapes = [(torch.bfloat16, 256, 8_000_000, False), (torch.bfloat16, 512, 8_000_000, False),
              (torch.bfloat16, 1024, 4_000_000, False), (torch.float16, 512, 8_000_000, False),
              (torch.bfloat16, 512, 8_000_000, True), (torch.bfloat16, 512, 86_567_656, False)]
    if os.environ.get("PROBE_BIGK"):
        shapes = [(torch.bfloat16, 1024, 4_000_000, False), (torch.bfloat16, 700, 4_000_000, False),
                  (torch.float16, 1024, 4_000_000, False), (torch.bfloat16, 1024, 4_000_000, True),
                  (torch.bfloat16, 1024, 43_283_828, False)]
    elif os.environ.get("PROBE_SMALLK"):
        shapes = [(torch.bfloat16, k, 8_000_000, False) for k in (16, 32, 48, 64, 96, 100, 128)]
        shapes += [(torch.bfloat16, 128, 8_000_000, True), (torch.bfloat16, 64, 86_567_656, False),
                   (torch.bfloat16, 128, 86_567_656, False)]
    elif os.environ.get("PROBE_QUICK"):
        shapes = shapes[1:2] + shapes[4:5] + (shapes[5:6] if os.environ.get("PROBE_QUICK") == "2" else [])
    for dtype, K, N, one_row in shapes:
        f16 = int(dtype == torch.float16)
        # one_row: every table entry points at row 0 (served from the caches): the selection's cost alone
        rows = rows_for(1 if one_row else K, N, dtype, dev, seed=K)
        tab = kn.upload_i64([rows[0 if one_row else i].data_ptr() for i in range(K)], dev)
        outs = {s: torch.empty(N, dtype=dtype, device=dev) for s in variants}
        ts = {s: [] for s in variants}
        for it in range(3 + reps):
            for s in variants:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(s, f16, tab, K, N, outs[s])
                b.record()
                b.synchronize()
                if it >= 3:
                    ts[s].append(a.elapsed_time(b))
        b1 = outs[variants[0]].view(torch.int16)
        diff = sum(int((b1 != outs[v].view(torch.int16)).sum()) for v in variants[1:])
        nbytes = (K + 1) * N * 2
        r = {"dtype": str(dtype)[6:], "K": K, "N": N, "one_row": one_row, "diff": diff}
        for s in variants:
            ms = statistics.median(ts[s])
            r[names[s]] = {"ms": round(ms, 4), "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}
        print(json.dumps(r), flush=True)
        res["timed"].append(r)
        assert diff == 0, r
        del rows, tab, outs
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
