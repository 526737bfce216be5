"""Where does per-client ingest time go? (tool)

Packs host clients (32 ResNet-50, or with --config cfg5 64 Llama-2-7B LoRA
updates of 16.8 MB) into pinned staging and sends them H2D under several
pipeline shapes; prints GB/s for each, plus the H2D alone from rotating
pre-packed pinned rows (the link at this copy size), with and without the
copy stream waiting on the current stream before each copy (what
ClientBucket does to order an H2D after earlier readers of the rows), and
the pack split into pieces whose H2Ds start as each piece is packed.

    python -m tools.ingest_probe [--config cfg5]
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3", choices=("cfg3", "cfg5"))
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K = 32 if a.config == "cfg3" else 64
    ents = [e for e in (shapes.resnet50() if a.config == "cfg3" else shapes.llama2_7b_lora()) if e[2] == torch.float32]
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

    def h2d_only(nbuf, wait):
        bufs = [torch.empty(L).pin_memory() for _ in range(nbuf)]
        st = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream()
        rates = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                if wait:
                    st.wait_stream(cur)
                with torch.cuda.stream(st):
                    rows[i].copy_(bufs[i % nbuf], non_blocking=True)
            torch.cuda.synchronize()
            rates.append(tot / (time.perf_counter() - t0) / 1e9)
        return max(rates)

    def pieces(nbuf, threads, P):
        """Each client packed in P pieces (by key), each piece's H2D issued as soon as it is packed."""
        bufs = [torch.empty(L).pin_memory() for _ in range(nbuf)]
        evs = [None] * nbuf
        st = torch.cuda.Stream(dev)
        cuts = []
        for srcs, offs, nbs, n in cl[:1]:
            per = max(1, n // P)
            cuts = [(j, min(n, j + per)) for j in range(0, n, per)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            b = i % nbuf
            if evs[b] is not None:
                evs[b].synchronize()
            srcs, offs, nbs, n = cl[i]
            for lo, hi in cuts:
                m = hi - lo
                sp = (ctypes.c_void_p * m)(*srcs[lo:hi])
                op = (ctypes.c_int64 * m)(*offs[lo:hi])
                np_ = (ctypes.c_int64 * m)(*nbs[lo:hi])
                lib.fedagg_host_pack(bufs[b].data_ptr(), sp, op, np_, m, threads)
                e0, e1 = offs[lo] // 4, (offs[hi - 1] + nbs[hi - 1]) // 4
                with torch.cuda.stream(st):
                    rows[i, e0:e1].copy_(bufs[b][e0:e1], non_blocking=True)
            with torch.cuda.stream(st):
                e = torch.cuda.Event()
                e.record(st)
            evs[b] = e
        torch.cuda.synchronize()
        return tot / (time.perf_counter() - t0) / 1e9

    print(f"{a.config}: {K} clients x {L * 4 / 1e6:.1f} MB", flush=True)
    for nbuf in (2, 3):
        print(f"H2D only, nbuf={nbuf}: {h2d_only(nbuf, False):6.1f} GB/s   with wait_stream before each copy: "
              f"{h2d_only(nbuf, True):6.1f} GB/s", flush=True)
    for P in (2, 4, 8):
        pieces(3, 16, P)
        print(f"pack + H2D in {P} pieces per client (nbuf=3, 16 threads): {pieces(3, 16, P):6.1f} GB/s", flush=True)
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
