"""A/B the fp32 weighted-sum kernel variants on the headline shape (GPU only).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24):
every variant runs once per round, R rounds, median/min reported.  Each
variant's output is checked bit-for-bit against a torch-on-GPU restatement of
the reference chain (separate mul and add kernels: two roundings, like the
reference's CPU loop).  Also times a plain device copy as the achievable-HBM
reference point.

    python tools/tune_wsum.py --K 128 --N 25610152 --rounds 10
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import _native as nat  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=25_610_152)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    K, N = a.K, a.N
    dev = torch.device("cuda:0")
    from tools import tuning_lib

    lib = tuning_lib.lib()  # the tuning build: the product library has no variant entries
    g = torch.Generator(device=dev).manual_seed(0)
    row = (N + 63) // 64 * 64
    bucket = torch.empty((K, row), dtype=torch.float32, device=dev)
    for i in range(K):
        bucket[i].normal_(0.0, 0.05, generator=g)
    n = torch.randint(100, 1001, (K,), generator=torch.Generator().manual_seed(1)).tolist()
    tot = sum(n)
    w = torch.tensor([float(x) / float(tot) for x in n], dtype=torch.float32, device=dev)
    ptrs = torch.tensor([bucket[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
    out = torch.empty(N, dtype=torch.float32, device=dev)
    st = nat.stream_handle()

    ref = None
    if not a.no_check:
        wl = w.cpu().tolist()
        ref = bucket[0, :N] * wl[0]
        for i in range(1, K):
            ref += bucket[i, :N] * wl[i]

    nv = lib.fedagg_num_variants()
    names = [lib.fedagg_variant_name(v).decode() for v in range(nv)]
    times = {nm: [] for nm in names}
    times["copy"] = []
    probe = None
    try:  # pure-read ceiling over the SAME 13 GB of rows, same process (tools/hbm_probe.hip)
        import ctypes
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        import hbm_probe
        probe = ctypes.CDLL(hbm_probe.build())
        probe.probe_read_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p]
        probe_out = torch.empty(8192 * 256, device=dev)
        times["read_probe"] = []
    except Exception as e:  # noqa: BLE001
        print("probe unavailable:", e)
    src_copy = bucket.view(-1)[: 8 * row].clone()
    dst_copy = torch.empty_like(src_copy)
    bytes_alg = (K + 1) * N * 4

    import ctypes
    hw = (ctypes.c_float * K)(*w.cpu().tolist()) if K <= 256 else None
    if hw is not None:  # the product entry with the weights in the kernel arguments (FedML's host weights)
        names.append("shipped_hostw")
        times["shipped_hostw"] = []

    def run(v: int) -> None:
        if v == nv:
            tuning_lib.check(lib.fedagg_wsum_f32(ptrs.data_ptr(), ctypes.addressof(hw), K, N, out.data_ptr(), 3, st),
                             "shipped_hostw")
            return
        tuning_lib.check(lib.fedagg_wsum_f32_variant(ptrs.data_ptr(), w.data_ptr(), K, N, out.data_ptr(), v, st),
                  names[v])

    for v in range(len(names)):  # warm-up + correctness
        run(v)
        torch.cuda.synchronize()
        if ref is not None:
            ok = torch.equal(out.view(torch.int32), ref.view(torch.int32))
            print(f"{names[v]}: bitwise={'OK' if ok else 'MISMATCH'}", flush=True)
            if not ok:
                d = (out - ref).abs().max().item()
                print(f"   max abs diff {d}", flush=True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for v in range(len(names)):
            ev0.record()
            run(v)
            ev1.record()
            ev1.synchronize()
            times[names[v]].append(ev0.elapsed_time(ev1))
        ev0.record()
        dst_copy.copy_(src_copy)
        ev1.record()
        ev1.synchronize()
        times["copy"].append(ev0.elapsed_time(ev1))
        if probe is not None:
            ev0.record()
            probe.probe_read_launch(bucket.data_ptr(), bucket.numel() // 4, probe_out.data_ptr(), 8192, 8, st)
            ev1.record()
            ev1.synchronize()
            times["read_probe"].append(ev0.elapsed_time(ev1))
    res = {}
    for nm, ts in times.items():
        med = statistics.median(ts)
        b = {"copy": 2 * src_copy.numel() * 4, "read_probe": bucket.numel() * 4}.get(nm, bytes_alg)
        res[nm] = {"median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                   "GBps_median": round(b / med / 1e6, 1), "frac_8TBps": round(b / med / 1e6 / 8000, 4)}
        print(f"{nm:10s} median {med:8.4f} ms  min {min(ts):8.4f} ms  {b / med / 1e6:8.1f} GB/s  "
              f"({b / med / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/tune_K{K}_N{N}.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
