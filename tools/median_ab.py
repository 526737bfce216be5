"""A/B two compile-time variants of csrc/median.hip in one process (tool only).

    python tools/median_ab.py [out.json]

Builds tools/_build/libmedian_{a,b}.so (MEDIAN_AB_DIR: another directory,
e.g. one that travels to the GPU box, built here beforehand with --build-only) from fedml_amd/csrc/median.hip with
the -D flags in VARIANTS (plus a stub for the library's error hook), loads
both, and times fedagg_median on the shapes below interleaved (2 warm-up, 9
timed launches each, HIP events on the launch stream); outputs must agree bit
for bit.  Rows as tools/median_bench.py.
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
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
# round 3: FEDAGG_PK16_MIRROR / FEDAGG_PK16_BATCH (profiles/r03/median_rsel/median_ab_pk16_merge.json); a
# 2-lanes-per-column split of 97..128 clients was 1.3-1.4x slower and was removed
# (median_ab_split128.json), so was sorting a K <= 128 column in two loaded-then-sorted halves
# (median_ab_halves.json); MEDIAN_AB_VARIANTS="tag=-DX=1,-DY=2;tag2=..." sets the variants
VARIANTS = {"new": ["-DFEDAGG_PK16_MIRROR=0"], "mirror": ["-DFEDAGG_PK16_MIRROR=1"]}
if os.environ.get("MEDIAN_AB_VARIANTS"):
    VARIANTS = {t: f.split(",") if f else [] for t, f in
                (v.split("=", 1) for v in os.environ["MEDIAN_AB_VARIANTS"].split(";"))}
STUB = 'extern "C" int fedagg_set_error_internal(int code, const char*) { return code; }\n'


def build():
    from fedml_amd import build as fb

    src = os.path.join(ROOT, "fedml_amd", "csrc", "median.hip")
    bdir = os.path.join(ROOT, os.environ.get("MEDIAN_AB_DIR", os.path.join("tools", "_build")))
    os.makedirs(bdir, exist_ok=True)
    stub = os.path.join(bdir, "median_ab_stub.cpp")
    open(stub, "w").write(STUB)
    procs, outs = [], {}
    for tag, flags in VARIANTS.items():
        so = os.path.join(bdir, f"libmedian_{tag}.so")
        outs[tag] = so
        if os.path.exists(so) and os.path.getmtime(so) > os.path.getmtime(src):
            continue
        procs.append(subprocess.Popen([fb.hipcc(), *fb.HIPCC_FLAGS, *flags, "-shared", "-o", so, src, stub]))
    for p in procs:
        assert p.wait() == 0
    return outs


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/median_ab.json"
    sos = build()
    if "--build-only" in sys.argv:
        return
    from fedml_amd import kernels as kn

    libs = {}
    for tag, so in sos.items():
        lib = ctypes.CDLL(so)
        lib.fedagg_median.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_void_p]
        libs[tag] = lib
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}  # FEDAGG_DT_*
    shapes = [(torch.bfloat16, 512, 4_000_036), (torch.bfloat16, 300, 4_000_036), (torch.bfloat16, 256, 4_000_036),
              (torch.float16, 512, 4_000_036), (torch.bfloat16, 512, 86_567_656)]
    if os.environ.get("MEDIAN_AB_SHAPES") == "k512":
        shapes = [(torch.float16, 512, 4_000_036), (torch.bfloat16, 512, 4_000_036), (torch.bfloat16, 300, 4_000_036),
                  (torch.bfloat16, 256, 4_000_036), (torch.float16, 512, 4_000_036), (torch.bfloat16, 512, 86_567_656)]
    if os.environ.get("MEDIAN_AB_SHAPES") == "lanes":  # both lane-group kernels (fp32 and packed 16-bit)
        shapes = [(torch.float32, 512, 4_000_037), (torch.bfloat16, 512, 4_000_036), (torch.float32, 300, 4_000_037),
                  (torch.bfloat16, 256, 4_000_036), (torch.bfloat16, 512, 86_567_656)]
    if os.environ.get("MEDIAN_AB_SHAPES") == "cols":  # the one-lane-per-column kernels (K <= 128)
        shapes = [(torch.float32, 128, 25_610_152), (torch.bfloat16, 128, 86_567_656), (torch.float32, 100, 25_610_152),
                  (torch.bfloat16, 64, 86_567_656)]
    shapes = [sh for sh in shapes if sh[2] <= int(os.environ.get("MEDIAN_AB_MAXN", "1000000000"))]
    reps = int(os.environ.get("MEDIAN_AB_REPS", "22"))
    res = []
    for dtype, K, N in shapes:
        L = (N + 63) // 64 * 64
        rows = torch.empty((K, L), dtype=dtype, device=dev)
        g = torch.Generator(device=dev).manual_seed(K)
        base = torch.randn(L, generator=g, device=dev) * 0.05
        for i in range(K):
            rows[i].copy_(base + 0.01 * torch.randn(L, generator=g, device=dev))
        del base
        tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
        outs = {t: torch.empty(L, dtype=dtype, device=dev) for t in libs}
        ts = {t: [] for t in libs}
        for rep in range(reps):
            order = list(libs.items())
            order = order[rep % len(order):] + order[:rep % len(order)]  # rotate who goes first
            for t, lib in order:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.fedagg_median(DT[dtype], tab.data_ptr(), K, N, outs[t].data_ptr(), 1, st)  # ALIGNED16
                e1.record()
                e1.synchronize()
                assert rc == 0, (t, rc)
                if rep >= min(2, reps - 1):
                    ts[t].append(e0.elapsed_time(e1))
        tags = list(libs)
        iv = torch.int32 if dtype == torch.float32 else torch.int16
        same = all(torch.equal(outs[tags[0]][:N].view(iv), outs[t][:N].view(iv)) for t in tags[1:])
        nbytes = (K + 1) * N * rows.element_size()
        r = {"dtype": str(dtype).replace("torch.", ""), "K": K, "N": N, "identical": bool(same)}
        for t in tags:
            ms = statistics.median(ts[t])
            r[f"{t}_ms"] = round(ms, 4)
            r[f"{t}_TBps"] = round(nbytes / (ms * 1e-3) / 1e12, 3)
        print(json.dumps(r), flush=True)
        res.append(r)
        del rows, outs
        torch.cuda.empty_cache()
    json.dump({"variants": VARIANTS, "results": res}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
