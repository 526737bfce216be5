"""A/B of two builds of libfedagg.so on the same buffers (tool only): the
fused FedAvg + server SGD / Adam steps of config 5 and the plain fp32 / bf16
FedAvg, each build's launch timed back to back (`--launches` per sample),
the builds interleaved round by round, medians reported.

    python tools/ab_libs.py fedml_amd/lib/ab/libfedagg_r05start.so fedml_amd/lib/libfedagg.so
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

P, I32, I64, U32, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    lib.fedagg_wsum_fedopt_sgd_f32.argtypes = [P, P, I32, I64, P, P, F, F, I32, U32, P]
    lib.fedagg_wsum_f32.argtypes = [P, P, I32, I64, P, U32, P]
    lib.fedagg_wsum_bf16.argtypes = [P, P, I32, I64, P, I32, U32, P]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = [load(p) for p in a.libs]
    st = nat.stream_handle()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cases = []
    # config 5: 64 x 4,194,304 fp32 + SGD (lr 1, momentum 0.9)
    K, N = 64, 4_194_304
    rows5 = torch.empty((K, N), device=dev).normal_(0.0, 0.05)
    p5 = torch.tensor([rows5[i].data_ptr() for i in range(K)], dtype=torch.int64, device=dev)
    w5 = torch.full((K,), 1.0 / K, device=dev)
    param = [torch.zeros(N, device=dev) for _ in libs]
    mom = [torch.zeros(N, device=dev) for _ in libs]
    cases.append(("cfg5 FedAvg+SGD", lambda i: libs[i].fedagg_wsum_fedopt_sgd_f32(
        p5.data_ptr(), w5.data_ptr(), K, N, param[i].data_ptr(), mom[i].data_ptr(), 1.0, 0.9, 0, 1, st)))
    hw = (ctypes.c_float * K)(*([1.0 / K] * K))  # FEDAGG_HOST_WEIGHTS: kernel-argument weights
    cases.append(("cfg5 SGD host-w", lambda i: libs[i].fedagg_wsum_fedopt_sgd_f32(
        p5.data_ptr(), ctypes.addressof(hw), K, N, param[i].data_ptr(), mom[i].data_ptr(), 1.0, 0.9, 0, 3, st)))
    out5 = [torch.empty(N, device=dev) for _ in libs]
    cases.append(("cfg5 FedAvg", lambda i: libs[i].fedagg_wsum_f32(p5.data_ptr(), w5.data_ptr(), K, N,
                                                                   out5[i].data_ptr(), 1, st)))
    # config 3's fp32 row
    K3, N3 = 128, 25_610_205
    L3 = (N3 + 63) // 64 * 64
    rows3 = torch.empty((K3, L3), device=dev).normal_(0.0, 0.05)
    p3 = torch.tensor([rows3[i].data_ptr() for i in range(K3)], dtype=torch.int64, device=dev)
    w3 = torch.full((K3,), 1.0 / K3, device=dev)
    out3 = [torch.empty(L3, device=dev) for _ in libs]
    cases.append(("cfg3 FedAvg", lambda i: libs[i].fedagg_wsum_f32(p3.data_ptr(), w3.data_ptr(), K3, N3,
                                                                   out3[i].data_ptr(), 1, st)))
    hw3 = (ctypes.c_float * K3)(*([1.0 / K3] * K3))
    cases.append(("cfg3 FedAvg host-w", lambda i: libs[i].fedagg_wsum_f32(p3.data_ptr(), ctypes.addressof(hw3), K3,
                                                                          N3, out3[i].data_ptr(), 3, st)))
    for name, fn in cases:
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
        print(f"{name:18s} {os.path.basename(a.libs[0])}: {m[0]:.4f} ms   {os.path.basename(a.libs[1])}: {m[1]:.4f} ms"
              f"   ({(m[1] / m[0] - 1) * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
