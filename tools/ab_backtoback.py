"""Back-to-back A/B of reduction tile shapes (tool only): each round times
`--launches` consecutive launches of one variant with two events around the
batch (the bench's regime: no idle gap between launches), variants interleaved
round by round, medians reported.  Variants come from the tuning table
(fedagg_wsum_tiny_variant) and are checked bit for bit against "shipped".

    python tools/ab_backtoback.py --dtype bf16 --K 512 --N 86567656 --variants shipped U4V4 U1V8 U2V4
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import _native as nat  # noqa: E402

# name -> (dtype code, row dtype, output dtype); bf16f32 = bf16 rows, fp32 partial out
DT = {"f32": (0, torch.float32, torch.float32), "bf16": (1, torch.bfloat16, torch.bfloat16),
      "bf16f32": (0x101, torch.bfloat16, torch.float32), "bf16acc32": (0x102, torch.bfloat16, torch.bfloat16)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=sorted(DT))
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--N", type=int, default=86_567_656)
    ap.add_argument("--variants", nargs="+", default=["shipped", "U4V4"])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--table", default="tiny", choices=["tiny", "f32"],
                    help="tiny: fedagg_wsum_tiny_variant (any --dtype); f32: fedagg_wsum_f32_variant (the fp32 "
                         "large-tile table: persistent, streaming, XCD forms)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from tools import tuning_lib

    lib = tuning_lib.lib()  # the tuning build: the product library has no variant entries
    if a.table == "f32":
        if a.dtype != "f32":
            raise SystemExit("--table f32 takes --dtype f32")
        names = [lib.fedagg_variant_name(v).decode() for v in range(lib.fedagg_num_variants())]
    else:
        names = [lib.fedagg_tiny_variant_name(v).decode() for v in range(lib.fedagg_num_tiny_variants())]
    idx = [names.index(v) for v in a.variants]
    code, dt, odt = DT[a.dtype]
    K, N = a.K, a.N
    L = (N + 63) // 64 * 64
    rows = torch.empty((K, L), device=dev, dtype=dt).normal_(0.0, 0.05)
    ptrs = torch.tensor([rows[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
    w = torch.rand(K, device=dev)
    w /= w.sum()
    outs = {v: torch.empty(L, device=dev, dtype=odt) for v in idx}
    st = nat.stream_handle()

    def run(v):
        if a.table == "f32":
            rc = lib.fedagg_wsum_f32_variant(ptrs.data_ptr(), w.data_ptr(), K, N, outs[v].data_ptr(), v, st)
        else:
            rc = lib.fedagg_wsum_tiny_variant(code, ptrs.data_ptr(), w.data_ptr(), K, N, outs[v].data_ptr(), v, st)
        tuning_lib.check(rc, names[v])

    for v in idx:
        run(v)
    torch.cuda.synchronize()
    ibits = torch.int16 if outs[idx[0]].element_size() == 2 else torch.int32
    ref = outs[idx[0]][:N].view(ibits)
    for v in idx:
        assert torch.equal(outs[v][:N].view(ibits), ref), names[v]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: [] for v in idx}
    for _ in range(a.rounds):
        for v in idx:
            run(v)
            ev0.record()
            for _ in range(a.launches):
                run(v)
            ev1.record()
            ev1.synchronize()
            times[v].append(ev0.elapsed_time(ev1) / a.launches)
    nbytes = K * N * rows.element_size() + N * outs[idx[0]].element_size()
    res = {names[v]: {"median_ms": statistics.median(t), "min_ms": min(t), "max_ms": max(t),
                      "GBps": nbytes / statistics.median(t) / 1e6} for v, t in times.items()}
    for n, r in res.items():
        print(f"{a.dtype} K={K} N={N} {n:14s} median {r['median_ms']:.4f} ms (min {r['min_ms']:.4f}, "
              f"max {r['max_ms']:.4f})  {r['GBps']:.0f} GB/s", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"K": K, "N": N, "dtype": a.dtype, "launches": a.launches, "rounds": a.rounds, "res": res}, f,
                      indent=1)


if __name__ == "__main__":
    main()
