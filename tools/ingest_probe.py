"""Where does per-client ingest time go? (tool)

Packs 32 ResNet-50 host clients into pinned staging and sends them H2D under
several pipeline shapes; prints GB/s for each.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import _native as nat  # noqa: E402
from fedml_amd import shapes  # noqa: E402
from tools.e2e_bench import make_clients  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    K = 32
    ents = [e for e in shapes.resnet50() if e[2] == torch.float32]
    raw = make_clients(ents, K, dev)
    L = shapes.numel(ents)
    rows = torch.empty((K, L), device=dev)
    lib = nat.lib()
    cl = []
    for _, d in raw:
        ts = list(d.values())
        offs, o = [], 0
        for t in ts:
            offs.append(o)
            o += t.numel() * 4
        n = len(ts)
        cl.append(((ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]), (ctypes.c_int64 * n)(*offs),
                   (ctypes.c_int64 * n)(*[t.numel() * 4 for t in ts]), n))
    tot = K * L * 4

    def run(nbuf, threads, use_stream=True):
        bufs = [torch.empty(L).pin_memory() for _ in range(nbuf)]
        evs = [None] * nbuf
        st = torch.cuda.Stream(dev) if use_stream else torch.cuda.current_stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp = 0.0
        for i in range(K):
            b = i % nbuf
            if evs[b] is not None:
                evs[b].synchronize()
            p0 = time.perf_counter()
            lib.fedagg_host_pack(bufs[b].data_ptr(), *cl[i], threads)
            tp += time.perf_counter() - p0
            with torch.cuda.stream(st):
                rows[i].copy_(bufs[b], non_blocking=True)
                e = torch.cuda.Event()
                e.record(st)
            evs[b] = e
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return tot / dt / 1e9, tot / tp / 1e9

    for nbuf in (1, 2, 3, 4):
        for th in (4, 8, 16):
            run(nbuf, th)
            r, p = run(nbuf, th)
            print(f"nbuf={nbuf} threads={th:2d}: ingest {r:6.1f} GB/s   (pack alone {p:6.1f} GB/s)", flush=True)
    # direct pageable per-key copies (no staging)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, (_, d) in enumerate(raw):
        o = 0
        for t in d.values():
            rows[i, o:o + t.numel()].copy_(t.reshape(-1), non_blocking=True)
            o += t.numel()
    torch.cuda.synchronize()
    print(f"per-key pageable copies: {tot / (time.perf_counter() - t0) / 1e9:6.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
