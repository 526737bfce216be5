"""End-to-end (host -> HBM -> host) rounds for any bench config (tool, GPU only).

    python tools/e2e_configs.py --config cfg5 [--distinct 8] [--rounds 3] [--out ...]

The north star's path starts and ends in host memory.  For the config's state
dict and client count (bench.CONFIGS), with pageable per-key host tensors as
unpickling produces them (`--distinct` different updates reused round-robin,
so config 4's 512 x 173 MB needs 1.4 GB of host memory, not 89 GB):

  xsilo      the cross-silo mirror (fedml_amd.cross_silo.FedMLAggregator):
             add_local_trained_result per arriving client (ingest into HBM),
             then check_whether_all_receive + aggregate() (the reduction over
             the device views; the result stays on the server device, as the
             reference's GPU server keeps it) and the copy of the averaged
             model to the host for the broadcast, per key (.cpu()) and by
             buffer (fedml_amd.host_copy.to_host, checked bit for bit);
             arrival GB/s, aggregate ms and round-end ms (aggregate +
             broadcast copy)
  agg_call   FedMLAggOperator.agg(args, host_list): the reference's call
             shape with the whole round inside one call; GB/s of host inputs
  link       pinned / pageable H2D and D2H ceilings of this box (1 GiB)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from fedml_amd import shapes  # noqa: E402
from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd.cross_silo import FedMLAggregator  # noqa: E402
from fedml_amd.host_copy import to_host  # noqa: E402
from fedml_amd.server_aggregator import MI355XServerAggregator  # noqa: E402
from fedml_amd.synth import sample_nums  # noqa: E402


class _Args:
    federated_optimizer = "FedAvg"


def make_updates(entries, D, dev):
    """D host state dicts: per-key pageable tensors of the model's dtypes,
    each with its own storage (generated on the GPU, copied down, every page
    touched)."""
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for i in range(D):
        d = OrderedDict()
        for k, s, dt in entries:
            if dt == torch.int64:
                d[k] = torch.full(s, 3 + i, dtype=torch.int64)
            else:
                d[k] = (torch.randn(s, generator=g, device=dev) * 0.05).to(dt).cpu()
        out.append(d)
    return out


def link(dev) -> dict:
    out = {}
    nb = 1 << 30
    pinned = torch.empty(nb // 4).pin_memory()
    pageable = torch.empty(nb // 4)
    pageable.fill_(1.0)
    d = torch.empty(nb // 4, device=dev)
    for name, fn in [("h2d_pinned_GBps", lambda: d.copy_(pinned, non_blocking=True)),
                     ("h2d_pageable_GBps", lambda: d.copy_(pageable)),
                     ("d2h_pinned_GBps", lambda: pinned.copy_(d, non_blocking=True))]:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out[name] = round(3 * nb / (time.perf_counter() - t0) / 1e9, 1)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5", choices=sorted(bench.CONFIGS))
    ap.add_argument("--distinct", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--agg-reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    entries = shapes.MODELS[cfg["model"]]()
    K = cfg["K"]
    ups = make_updates(entries, a.distinct, dev)
    ns = sample_nums(K)
    nbytes = sum(t.numel() * t.element_size() for t in ups[0].values())
    res = {"config": a.config, "workload": cfg["desc"], "clients": K, "bytes_per_client": nbytes,
           "host_bytes_per_round": K * nbytes, "distinct_updates": a.distinct, "link": link(dev)}
    print(json.dumps(res), flush=True)

    # the cross-silo mirror: arrival ingest, round-end aggregate()
    args = _Args()
    agg = MI355XServerAggregator(torch.nn.Linear(1, 1), args)
    agg.set_model_params = lambda p: None  # the server model is a stand-in (no torchvision here)
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, dev, args, agg)
    rounds = []
    for r in range(a.rounds + 1):  # round 0 builds the bucket and the pinned staging
        per = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            s = time.perf_counter()
            server.add_local_trained_result(i, OrderedDict(ups[i % a.distinct]), ns[i])
            per.append(time.perf_counter() - s)
        t1 = time.perf_counter()
        server.check_whether_all_receive()
        averaged, _, _ = server.aggregate()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host = OrderedDict((k, t.cpu()) for k, t in averaged.items())  # the broadcast's copy to the host
        t3 = time.perf_counter()
        assert all(not t.is_cuda for t in host.values())
        host2 = to_host(averaged)  # the same copy, one DMA per result buffer (fedml_amd.host_copy)
        t4 = time.perf_counter()
        assert all(torch.equal(host[k].view(-1).view(torch.uint8), host2[k].view(-1).view(torch.uint8))
                   for k in host)
        if r:
            rounds.append({"arrival_ms_median": round(statistics.median(per) * 1e3, 3),
                           "arrival_GBps": round(nbytes / statistics.median(per) / 1e9, 1),
                           "all_arrivals_s": round(t1 - t0, 4),
                           "ingest_GBps": round(K * nbytes / (t1 - t0) / 1e9, 1),
                           "aggregate_ms": round((t2 - t1) * 1e3, 2),
                           "broadcast_d2h_ms": round((t3 - t2) * 1e3, 2),
                           "broadcast_to_host_ms": round((t4 - t3) * 1e3, 2),
                           "round_end_ms": round((t3 - t1) * 1e3, 2),
                           "round_end_to_host_ms": round((t2 - t1 + t4 - t3) * 1e3, 2)})
        print(a.config, "xsilo round", r, rounds[-1] if r else "(warm-up)", flush=True)
        time.sleep(0.2)  # the next round's arrivals, in which the result pool refills
    res["xsilo"] = {"rounds": rounds,
                    "round_end_ms_median": statistics.median(x["round_end_ms"] for x in rounds),
                    "round_end_to_host_ms_median": statistics.median(x["round_end_to_host_ms"] for x in rounds),
                    "ingest_GBps_median": statistics.median(x["ingest_GBps"] for x in rounds)}
    del server, agg
    torch.cuda.empty_cache()

    # the reference's call shape: the whole round in one agg() call
    ts = []
    for r in range(a.agg_reps + 1):
        lst = [(ns[i], OrderedDict(ups[i % a.distinct])) for i in range(K)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = FedMLAggOperator.agg(_Args(), lst)
        torch.cuda.synchronize()
        if r:
            ts.append(time.perf_counter() - t0)
        assert all(not t.is_cuda for t in out.values())
        print(a.config, "agg() call", r, round(time.perf_counter() - t0, 4), flush=True)
    med = statistics.median(ts)
    res["agg_call"] = {"s_median": round(med, 4), "host_GBps": round(K * nbytes / med / 1e9, 1),
                       "all_s": [round(x, 4) for x in ts]}
    print(json.dumps(res, indent=1))
    out = a.out or os.path.join("gpurun_out", f"e2e_{a.config}.json")
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
