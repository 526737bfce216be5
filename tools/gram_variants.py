"""A/B of compile-time variants of the centred-Gram Krum kernel (tool only).

    python tools/gram_variants.py --build      # CPU container: tools/_build/robust_<tag>.so
    python tools/gram_variants.py --rounds 9   # GPU box

Each variant is csrc/robust.hip built standalone with its -D flags (plus a
stub for the error hook it takes from fedagg.hip).  fedagg_pairgram2_f32 at
config 3 (128 clients x ResNet-50's weights, base + 0.01 noise per client as
bench.py), variants interleaved in one process, HIP events on the launch
stream, outputs compared bit for bit.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, os.environ.get("GRAM_AB_DIR", os.path.join("tools", "_build")))
# tag -> -D flags of the knobs under test (none are left in robust.hip: the
# round-3 probes of a swizzled 72-float LDS row and of block-pipelined
# fragment reads were bit-identical and slower, 5.97 and 8.49 ms against
# 5.79 ms; profiles/r03/dist/gram_variants.txt).  Extra variants: --variant
# TAG=-DFLAG=V,-DFLAG2=V2
VARIANTS = {"same": []}
STUB = 'extern "C" int fedagg_set_error_internal(int code, const char*) { return code; }\n'


def build() -> None:
    from fedml_amd import build as fb

    os.makedirs(OUT, exist_ok=True)
    stub = os.path.join(OUT, "stub.cpp")
    open(stub, "w").write(STUB)
    src = os.path.join(ROOT, "fedml_amd", "csrc", "robust.hip")
    procs = [subprocess.Popen([fb.hipcc(), *fb.HIPCC_FLAGS, *flags, "-shared", "-o",
                               os.path.join(OUT, f"robust_{tag}.so"), src, stub]) for tag, flags in VARIANTS.items()]
    assert all(p.wait() == 0 for p in procs)


def bench(rounds: int, out_path: str, chunk: int = 0) -> None:
    import torch

    from fedml_amd import _native as nat
    from fedml_amd import defense as dfn
    from fedml_amd import shapes
    from fedml_amd.bucket import ClientBucket

    dev = torch.device("cuda:0")
    K = 128
    b = ClientBucket(shapes.resnet50(), K, dev)
    g = b.groups[torch.float32]
    gen = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(g.rows.shape[1], generator=gen, device=dev) * 0.05
    for i in range(K):
        g.rows[i].copy_(base + 0.01 * torch.randn(g.rows.shape[1], generator=gen, device=dev))
    del base
    chunks, n_chunks = dfn.weight_chunks(g, nat.DIST_CHUNK, dev)
    work = dfn._work(nat.WORK_PAIRGRAM, K, n_chunks, dev)
    st = nat.stream_handle()
    libs = {"shipped": nat.lib()}
    for tag in VARIANTS:
        libs[tag] = ctypes.CDLL(os.path.join(OUT, f"robust_{tag}.so"))
    outs = {t: torch.empty((K, K), dtype=torch.float64, device=dev) for t in libs}
    times = {t: [] for t in libs}
    stamps = {}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tags = list(libs)
    for r in range(rounds + 1):
        order = tags[r % len(tags):] + tags[:r % len(tags)]
        for tag in order:
            lib = libs[tag]
            ev0.record()
            rc = lib.fedagg_pairgram2_f32(ctypes.c_void_p(g.d_ptrs.data_ptr()), K, ctypes.c_void_p(chunks.data_ptr()),
                                          ctypes.c_int64(n_chunks), ctypes.c_void_p(outs[tag].data_ptr()),
                                          ctypes.c_void_p(work.data_ptr()), ctypes.c_int64(work.numel()),
                                          ctypes.c_void_p(st))
            ev1.record()
            ev1.synchronize()
            assert rc == 0, tag
            if r:
                times[tag].append(ev0.elapsed_time(ev1))
            if tag.startswith("stamps") and r == rounds:
                # FEDAGG_GRAM_STAMPS: blocks 0..7 x 8 waves x 4 phases (split +
                # fetch, MFMAs, sums, barrier) in s_memtime ticks summed over
                # 128 iterations, after the 256 used blocks' partials
                nt = ((K + 15) // 16) * ((K + 15) // 16 + 1) // 2
                stt = work[256 * nt * 256: 256 * nt * 256 + 8 * 8 * 4].view(8, 8, 4).cpu() / 128
                stamps[tag] = {"per_wave_mean_ticks": [[round(float(x), 1) for x in stt[:, w, :].mean(0)]
                                                       for w in range(8)],
                               "phases": ["split+fetch", "mfma", "sums", "barrier"]}
                print(tag, stamps[tag], flush=True)
    # the exact-difference kernel's D, and each variant's error against it in
    # the units test_gpu_dist_defenses.py bounds (|c_i|^2 + |c_j|^2, the
    # double-centred norms)
    exact = torch.empty((K, K), dtype=torch.float64, device=dev)
    wex = dfn._work(nat.WORK_PAIRDIST2, K, n_chunks, dev)
    assert nat.lib().fedagg_pairdist2_f32(ctypes.c_void_p(g.d_ptrs.data_ptr()), K, ctypes.c_void_p(chunks.data_ptr()),
                                          ctypes.c_int64(n_chunks), ctypes.c_void_p(exact.data_ptr()),
                                          ctypes.c_void_p(wex.data_ptr()), ctypes.c_int64(wex.numel()),
                                          ctypes.c_void_p(st)) == 0
    torch.cuda.synchronize()
    cn = exact.mean(1) - exact.sum() / (2 * K * K)
    scale = cn[:, None] + cn[None, :]
    off = ~torch.eye(K, dtype=torch.bool, device=dev)
    res = {"K": K, "n_chunks": int(n_chunks), "chunk": chunk or nat.PAIR_CHUNK, "variants": VARIANTS}
    for tag in tags:
        err = ((outs[tag] - exact).abs() / scale)[off]
        res[tag] = {"ms": round(statistics.median(times[tag]), 4),
                    "identical_to_shipped": bool(torch.equal(outs[tag], outs["shipped"])),
                    "max_err_vs_exact": float(err.max()),
                    "krum_order_same_as_exact": bool(torch.equal(outs[tag].sort(1).values[:, :64].sum(1).argsort(),
                                                                 exact.sort(1).values[:, :64].sum(1).argsort()))}
        print(tag, res[tag], flush=True)
    res["stamps"] = stamps
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--out", default="gpurun_out/gram_variants.json")
    ap.add_argument("--variant", action="append", default=[], help="TAG=-DFLAG=V[,-DFLAG2=V2]")
    ap.add_argument("--chunk", type=int, default=0, help="chunk-table piece length (default FEDAGG_PAIR_CHUNK)")
    a = ap.parse_args()
    for v in a.variant:
        tag, flags = v.split("=", 1)
        VARIANTS[tag] = flags.split(",")
    if a.build:
        build()
    else:
        bench(a.rounds, a.out, a.chunk)
