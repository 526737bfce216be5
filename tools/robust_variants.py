"""A/B of compile-time variants of csrc/robust.hip (GPU only for the timing).

Builds csrc/robust.hip standalone into tools/_build/robust_<tag>.so once per
-D setting (with a stub for the one symbol it takes from fedagg.hip), then
times the clipped rebuild and the distance kernels of each build at config 3
(128 clients x ResNet-50's fp32 row), interleaved in one process, every
variant checked bit for bit against the library's own result.

    python tools/robust_variants.py --build          # CPU container
    python tools/robust_variants.py --rounds 10      # GPU box
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
VARIANTS = {"clip1": ["-DFEDAGG_CLIP_CLIENTS=1"], "clip4": ["-DFEDAGG_CLIP_CLIENTS=4"],
            "d16nt": ["-DFEDAGG_DIST2_REF_NT=true"], "d32": ["-DFEDAGG_DIST2_BATCH=32"]}
if os.environ.get("ROBUST_VARIANTS"):  # "tag=-DX=1,-DY=2;tag2=..."
    VARIANTS = {t: f.split(",") if f else [] for t, f in
                (v.split("=", 1) for v in os.environ["ROBUST_VARIANTS"].split(";"))}
STUB = 'extern "C" int fedagg_set_error_internal(int code, const char*) { return code; }\n'


def build() -> None:
    from fedml_amd import build as fb

    os.makedirs(OUT, exist_ok=True)
    stub = os.path.join(OUT, "stub.cpp")
    with open(stub, "w") as f:
        f.write(STUB)
    src = os.path.join(ROOT, "fedml_amd", "csrc", "robust.hip")
    for tag, flags in VARIANTS.items():
        so = os.path.join(OUT, f"robust_{tag}.so")
        cmd = [fb.hipcc(), *fb.HIPCC_FLAGS, *flags, "-shared", "-o", so, src, stub]
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)


def bench(rounds: int) -> None:
    import torch

    from fedml_amd import _native as nat
    from fedml_amd import kernels as kn
    from fedml_amd import shapes
    from fedml_amd.bucket import ClientBucket

    dev = torch.device("cuda:0")
    K = 128
    b = ClientBucket(shapes.resnet50(), K, dev)
    g = b.groups[torch.float32]
    gen = torch.Generator(device=dev).manual_seed(0)
    g.rows.normal_(0.0, 0.05, generator=gen)
    ref = g.rows[K - 1].clone()
    out = torch.empty_like(g.rows)
    d_dst = kn.upload_i64([out[i].data_ptr() for i in range(K)], dev)
    d_div = kn.upload_f32([1.0 + 0.01 * (i % 3) for i in range(K)], dev)
    st = nat.stream_handle()
    libs = {} if os.environ.get("ROBUST_NO_SHIPPED") else {"shipped": nat.lib()}
    for tag in VARIANTS:
        libs[tag] = ctypes.CDLL(os.path.join(OUT, f"robust_{tag}.so"))
    want = None
    times = {t: [] for t in libs}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds + 1):
        for tag, lib in libs.items():
            ev0.record()
            rc = lib.fedagg_clip_diff_f32(ctypes.c_void_p(g.d_ptrs.data_ptr()), K, ctypes.c_void_p(ref.data_ptr()),
                                          ctypes.c_void_p(d_div.data_ptr()), ctypes.c_int64(g.length),
                                          ctypes.c_void_p(d_dst.data_ptr()), ctypes.c_void_p(st))
            ev1.record()
            ev1.synchronize()
            assert rc == 0, tag
            if r == 0:
                if want is None:
                    want = out.clone()
                else:
                    assert torch.equal(out.view(torch.int32), want.view(torch.int32)), tag
                continue
            times[tag].append(ev0.elapsed_time(ev1))
    alg = (2 * K + 1) * g.length * 4
    for tag, ts in times.items():
        m = statistics.median(ts)
        print(f"clip {tag:8s} median {m:.4f} ms  {alg / m / 1e6:7.1f} GB/s  ({alg / m / 1e6 / 8000:.3f})", flush=True)
    # the read + write ceiling for the clip: a device copy of the same bytes
    ct = []
    for _ in range(rounds):
        ev0.record()
        out.copy_(g.rows)
        ev1.record()
        ev1.synchronize()
        ct.append(ev0.elapsed_time(ev1))
    m = statistics.median(ct)
    cb = 2 * g.rows.numel() * 4
    print(f"copy     median {m:.4f} ms  {cb / m / 1e6:7.1f} GB/s  ({cb / m / 1e6 / 8000:.3f}) [same rows, read + write]")
    # dist2 (every client's distance to a reference row), all builds
    from fedml_amd import defense as dfn

    chunks, n_chunks = dfn.weight_chunks(g, nat.DIST_CHUNK, dev)
    d_out = torch.empty(K, dtype=torch.float64, device=dev)
    work = dfn._work(nat.WORK_DIST2, K, n_chunks, dev)
    n_w = sum(n for k, n in zip(g.keys, g.numels) if dfn.is_weight_param(k))
    dt = {t: [] for t in libs}
    want = None
    for r in range(rounds + 1):
        for tag, lib in libs.items():
            ev0.record()
            rc = lib.fedagg_dist2_f32(ctypes.c_void_p(g.d_ptrs.data_ptr()), K, ctypes.c_void_p(ref.data_ptr()),
                                      ctypes.c_void_p(chunks.data_ptr()), ctypes.c_int64(n_chunks),
                                      ctypes.c_void_p(d_out.data_ptr()), ctypes.c_void_p(work.data_ptr()),
                                      ctypes.c_int64(work.numel()), ctypes.c_void_p(st))
            ev1.record()
            ev1.synchronize()
            assert rc == 0, tag
            if r == 0:
                if want is None:
                    want = d_out.clone()
                else:
                    assert torch.allclose(d_out, want, rtol=1e-13), tag
                continue
            dt[tag].append(ev0.elapsed_time(ev1))
    alg = (K + 1) * n_w * 4
    for tag, ts in dt.items():
        m = statistics.median(ts)
        print(f"dist2 {tag:8s} median {m:.4f} ms  {alg / m / 1e6:7.1f} GB/s  ({alg / m / 1e6 / 8000:.3f})", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        bench(a.rounds)
