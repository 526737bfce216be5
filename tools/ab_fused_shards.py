"""A/B of two builds of libfedagg.so on the fused FedOpt kernels at the sizes a
device sees when a config-5 round (and, for reference, the plain FedAvg there) (64 clients x 4,194,304 fp32 LoRA
parameters) is split over G = 8 / 4 / 2 / 1 GPUs (tool only).  Each build's
launch is timed back to back (`--launches` per sample), the builds interleaved
round by round, medians reported with the HBM rate of the algorithmic bytes.

    python tools/ab_fused_shards.py tools/_abbuild/libfedagg_before.so fedml_amd/lib/libfedagg.so
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import _native as nat  # noqa: E402

HOST_W = 3  # FEDAGG_HOST_WEIGHTS | FEDAGG_ALIGNED16: the weights in the kernel arguments, as FedOptServer passes them


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in nat.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = [load(p) for p in a.libs]
    st = nat.stream_handle()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K, N_full = 64, 4_194_304
    rows = torch.empty((K, N_full), device=dev).normal_(0.0, 0.05)
    hw = (ctypes.c_float * K)(*([1.0 / K] * K))
    sc9 = (ctypes.c_float * 9)()
    carry = (ctypes.c_float * 2)(1.0, 1.0)
    nat.check(libs[1].fedagg_optrepo_scalars(1, 1e-3, 5, carry, sc9), "scalars")
    sc6 = (ctypes.c_float * 6)()
    nat.check(libs[1].fedagg_adam_scalars(1e-3, 0.9, 0.999, 1e-8, 5, sc6), "adam scalars")
    for G in (8, 4, 2, 1):
        N = N_full // G
        ptrs = torch.tensor([rows[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
        param = [torch.zeros(N, device=dev) for _ in libs]
        s0 = [torch.zeros(N, device=dev) for _ in libs]
        s1 = [torch.ones(N, device=dev) for _ in libs]
        w = ctypes.addressof(hw)
        out = [torch.empty(N, device=dev) for _ in libs]
        cases = {
            "avg": (4 * K * N + 4 * N, lambda i: libs[i].fedagg_wsum_f32(
                ptrs.data_ptr(), w, K, N, out[i].data_ptr(), HOST_W, st)),
            "sgd": (4 * K * N + 16 * N, lambda i: libs[i].fedagg_wsum_fedopt_sgd_f32(
                ptrs.data_ptr(), w, K, N, param[i].data_ptr(), s0[i].data_ptr(), 1.0, 0.9, 0, HOST_W, st)),
            "adam": (4 * K * N + 24 * N, lambda i: libs[i].fedagg_wsum_fedopt_adam_f32(
                ptrs.data_ptr(), w, K, N, param[i].data_ptr(), s0[i].data_ptr(), s1[i].data_ptr(), sc6, 0, HOST_W,
                st)),
            "adamax": (4 * K * N + 24 * N, lambda i: libs[i].fedagg_wsum_fedopt_optrepo_f32(
                1, ptrs.data_ptr(), w, K, N, param[i].data_ptr(), s0[i].data_ptr(), s1[i].data_ptr(), sc9, HOST_W,
                st)),
        }
        for name, (alg, fn) in cases.items():
            for i in range(2):
                nat.check(fn(i), name)
            torch.cuda.synchronize()
            times = [[], []]
            for _ in range(a.rounds):
                for i in range(2):
                    ev0.record()
                    for _ in range(a.launches):
                        fn(i)
                    ev1.record()
                    ev1.synchronize()
                    times[i].append(ev0.elapsed_time(ev1) / a.launches)
            m = [statistics.median(t) for t in times]
            same = torch.equal(out[0], out[1]) if name == "avg" else (
                torch.equal(param[0], param[1]) and torch.equal(s0[0], s0[1]))
            print(f"G={G} N={N:>9,} {name:7s} A {m[0] * 1e3:7.1f} us ({alg / (m[0] * 1e-3) / 1e9 / 8000:.3f} of HBM)   "
                  f"B {m[1] * 1e3:7.1f} us ({alg / (m[1] * 1e-3) / 1e9 / 8000:.3f} of HBM)   {(m[1] / m[0] - 1) * 100:+.1f} %   "
                  f"bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
