"""Many clients over small tensors (the cross-device shape): 16-byte tiles
against narrow packs (reduce_narrow_kernel, EL elements per lane, U clients in
flight), fp32 and bf16 (reference chain), GPU only.  Every variant is checked
bit for bit against the shipped dispatch; median of R interleaved rounds.

    python tools/tune_tiny.py --rounds 15 > gpurun_out/tune_tiny.txt
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

DT = {"f32": (0, torch.float32), "bf16": (1, torch.bfloat16)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--dtypes", nargs="*", default=["f32", "bf16"])
    ap.add_argument("--K", type=int, nargs="*", default=[48, 128, 1000, 4096])
    ap.add_argument("--N", type=int, nargs="*", default=[7850, 62006, 200000, 1000000])
    ap.add_argument("--out", default="gpurun_out/tune_tiny.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from tools import tuning_lib

    lib = tuning_lib.lib()  # the tuning build: the product library has no variant entries
    names = [lib.fedagg_tiny_variant_name(v).decode() for v in range(lib.fedagg_num_tiny_variants())]
    st = nat.stream_handle()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for dname in a.dtypes:
        code, dt = DT[dname]
        esz = torch.empty((), dtype=dt).element_size()
        for K in a.K:
            for N in a.N:
                L = (N + 63) // 64 * 64
                rows = torch.empty((K, L), device=dev, dtype=dt).normal_(0.0, 0.05)
                ptrs = torch.tensor([rows[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
                w = torch.rand(K, device=dev)
                w /= w.sum()
                outs = [torch.empty(L, device=dev, dtype=dt) for _ in names]
                times = [[] for _ in names]

                def run(v):
                    tuning_lib.check(lib.fedagg_wsum_tiny_variant(code, ptrs.data_ptr(), w.data_ptr(), K, N,
                                                           outs[v].data_ptr(), v, st), names[v])

                for v in range(len(names)):
                    run(v)
                torch.cuda.synchronize()
                ref = outs[0][:N].view(torch.int16 if esz == 2 else torch.int32)
                for v in range(len(names)):
                    got = outs[v][:N].view(torch.int16 if esz == 2 else torch.int32)
                    assert torch.equal(got, ref), (dname, K, N, names[v])
                for _ in range(a.rounds):
                    for v in range(len(names)):
                        ev0.record()
                        run(v)
                        ev1.record()
                        ev1.synchronize()
                        times[v].append(ev0.elapsed_time(ev1))
                med = {names[v]: statistics.median(times[v]) for v in range(len(names))}
                best = min(med, key=med.get)
                gbs = {n: K * N * esz / m / 1e6 for n, m in med.items()}
                res[f"{dname}_K{K}_N{N}"] = {"median_ms": med, "GBps": gbs, "best": best}
                print(f"{dname:4s} K={K:5d} N={N:8d} best {best:9s} {med[best]:.4f} ms {gbs[best]:6.0f} GB/s "
                      f"(shipped {med['shipped']:.4f}) | " + " ".join(f"{n}={m:.4f}" for n, m in med.items()),
                      flush=True)
                del rows, ptrs, outs
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
