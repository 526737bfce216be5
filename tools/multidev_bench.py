"""Cost of spreading one round over G devices in ONE process (fedml_amd.multidev),
measured with the G shards on the box's one GPU (GPU only).

Two call shapes at config 3's state dict (ResNet-50, 320 keys, int64
counters), K clients:

  host   FedMLAggOperator.agg(args, host dicts) with args.fedagg_devices listing
         G devices: per-shard pack + H2D, per-shard reduction, per-shard D2H and
         scatter into per-key host tensors (FedML's CPU-server call shape);
  device the cross-silo shape: each client's dict rebound to views of its
         slot in a MultiDeviceBucket, then agg() on the views (the walker
         groups the keys by device and launches each device's chunks).

On one GPU the shards share one PCIe link and one HBM, so this measures the
splitting overhead (more launches, copies, streams), not the G-fold bandwidth
of G GPUs.  Every G's result is compared bit for bit with G = 1.

    python tools/multidev_bench.py --clients 32 --reps 3
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import agg_operator as ao  # noqa: E402
from fedml_amd import shapes  # noqa: E402
from fedml_amd.multidev import MultiDeviceBucket  # noqa: E402


class Args:
    federated_optimizer = "FedAvg"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shards", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--out", default="gpurun_out/r04/multidev_bench.json")
    ap.add_argument("--ingest", action="store_true",
                    help="also time put() x K + reduce_to_host on resident buckets, the G values interleaved")
    ap.add_argument("--shared-copy", action="store_true",
                    help="--ingest: add arms where every shard of G > 1 stages on ONE shared copy stream")
    ap.add_argument("--ab-pack", action="store_true",
                    help="host rounds: time the pack pool and round 3's threads per call, interleaved")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    entries = shapes.resnet50()
    K = a.clients
    g = torch.Generator(device=dev).manual_seed(0)
    raw = []
    for i in range(K):
        d = OrderedDict()
        for k, s, dt in entries:
            if dt == torch.int64:
                d[k] = torch.full(s, 5 + i, dtype=dt)
            else:
                d[k] = (torch.randn(s, generator=g, device=dev) * 0.05).cpu()
        raw.append((100 + 7 * i, d))
    nbytes = K * sum(t.numel() * t.element_size() for t in raw[0][1].values())
    res = {"clients": K, "model": "resnet50", "host_bytes_per_round": nbytes, "host": {}, "device": {}}
    ref_host = None
    modes = ["pool", "spawn"] if a.ab_pack else ["pool"]
    for G in a.shards:
        args = Args()
        args.fedagg_devices = [dev] * G
        ts = []
        tmode = {m: [] for m in modes}
        out = None
        for r in range(a.reps + 1):
            order = modes[r % len(modes):] + modes[:r % len(modes)]
            for m in order:  # --ab-pack: the native pack's pool vs round 3's threads per call, interleaved
                os.environ["FEDAGG_PACK_SPAWN"] = "1" if m == "spawn" else "0"
                lst = [(n, OrderedDict(d)) for n, d in raw]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = ao.FedMLAggOperator.agg(args, lst)
                torch.cuda.synchronize()
                if r:
                    tmode[m].append(time.perf_counter() - t0)
        os.environ["FEDAGG_PACK_SPAWN"] = "0"
        ts = tmode["pool"]
        if a.ab_pack:
            res.setdefault("host_spawn_ms", {})[f"G{G}"] = round(statistics.median(tmode["spawn"]) * 1e3, 2)
        if ref_host is None:
            ref_host = out
        same = all(torch.equal(out[k].view(-1).view(torch.int32) if out[k].dtype == torch.float32 else out[k],
                               ref_host[k].view(-1).view(torch.int32) if ref_host[k].dtype == torch.float32
                               else ref_host[k]) for k in out)
        ms = statistics.median(ts) * 1e3
        res["host"][f"G{G}"] = {"ms": round(ms, 2), "GBps_host_in": round(nbytes / ms / 1e6, 1),
                                "bitwise_equal_to_G1": same}
        print("host", G, res["host"][f"G{G}"], flush=True)
        ao._MULTI.clear()
        ao._BUCKETS.clear()
    ref_dev = None
    for G in a.shards:
        b = MultiDeviceBucket([(k, s, dt) for k, s, dt in entries], K, [dev] * G, promote_ints=False)
        views = []
        for i, (n, d) in enumerate(raw):
            b.put(i, d, n)
            views.append((n, b.view(i)))
        b.sync_ingest()
        torch.cuda.synchronize()
        ts = []
        out = None
        for r in range(a.reps * 3 + 1):
            lst = [(n, OrderedDict(v)) for n, v in views]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = ao.FedMLAggOperator.agg(Args(), lst)
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t0)
        if ref_dev is None:
            ref_dev = OrderedDict((k, t.clone()) for k, t in out.items())
        same = all(torch.equal(out[k], ref_dev[k]) for k in out)
        ms = statistics.median(ts) * 1e3
        res["device"][f"G{G}"] = {"ms": round(ms, 3), "bitwise_equal_to_G1": same}
        print("device", G, res["device"][f"G{G}"], flush=True)
        del b, views, out
        torch.cuda.empty_cache()
    if a.ingest:
        # the cross-silo arrival path: every client put() into resident
        # buckets (one per arm, built once), then reduce_to_host; the arms
        # interleaved per round in this one process, so host drift cancels.
        # --shared-copy adds "G<n>s" arms whose shards all stage on ONE copy
        # stream: if G shards on one GPU cost more only because their copy
        # streams contend for the one PCIe link, a shared stream (strictly
        # serial copies) should cost no more than the per-shard streams
        arms = {f"G{G}": G for G in a.shards}
        if a.shared_copy:
            arms.update({f"G{G}s": G for G in a.shards if G > 1})
        buckets = {}
        for name, G in arms.items():
            b = MultiDeviceBucket([(k, s, dt) for k, s, dt in entries], K, [dev] * G)
            if name.endswith("s"):
                shared = torch.cuda.Stream(dev)
                for sh in b.shards:
                    sh._copy = shared
            buckets[name] = b
        ns = [n for n, _ in raw]
        names = list(arms)
        tin = {n: [] for n in names}
        outs = {}
        for r in range(a.reps * 2 + 1):
            order = names[r % len(names):] + names[:r % len(names)]
            for name in order:
                b = buckets[name]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i, (n, d) in enumerate(raw):
                    b.put(i, d, n)
                outs[name] = b.reduce_to_host(b.weights(ns))
                torch.cuda.synchronize()
                if r:
                    tin[name].append(time.perf_counter() - t0)
        g0 = names[0]
        res["ingest"] = {}
        for name in names:
            same = all(torch.equal(outs[name][k].view(-1).view(torch.int32) if outs[name][k].dtype == torch.float32
                                   else outs[name][k], outs[g0][k].view(-1).view(torch.int32)
                                   if outs[g0][k].dtype == torch.float32 else outs[g0][k]) for k in outs[g0])
            ms = statistics.median(tin[name]) * 1e3
            res["ingest"][name] = {"ms": round(ms, 2), "GBps_host_in": round(nbytes / ms / 1e6, 1),
                                   "vs_G1": round(ms / (statistics.median(tin[g0]) * 1e3), 4),
                                   "all_ms": [round(x * 1e3, 2) for x in tin[name]],
                                   "shared_copy_stream": name.endswith("s"), "bitwise_equal_to_G1": same}
            print("ingest", name, res["ingest"][name], flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
