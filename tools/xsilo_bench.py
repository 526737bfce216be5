"""Cross-silo server round at config 3 (128 clients x ResNet-50 state dicts
arriving from the host one at a time), through fedml_amd.cross_silo's
FedMLAggregator: per-client arrival cost (ingest into HBM) and the round-end
aggregate().  Beside it, the reference's flow on the same GPU: per-key
`.to(device)` at arrival (model_params_to_device, ml_engine_adapter.py:234-254)
and the eager torch_aggregator loop (agg_operator.py:35-44) at round end.

    python tools/xsilo_bench.py [--K 128] [--distinct 8]
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

from fedml_amd import shapes  # noqa: E402
from fedml_amd.cross_silo import FedMLAggregator  # noqa: E402
from fedml_amd.server_aggregator import MI355XServerAggregator  # noqa: E402
from fedml_amd.synth import host_clients, sample_nums  # noqa: E402


class _Args:
    federated_optimizer = "FedAvg"


def _eager_fedavg(raw):
    """The reference's FedAvg loop (agg_operator.py:35-44), torch eager."""
    training_num = sum(n for n, _ in raw)
    (num0, avg) = raw[0]
    for k in avg.keys():
        for i in range(len(raw)):
            n, p = raw[i]
            w = n / training_num
            if i == 0:
                avg[k] = p[k] * w
            else:
                avg[k] += p[k] * w
    return avg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--distinct", type=int, default=8, help="distinct host updates, reused round-robin")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    entries = shapes.resnet50()
    base = host_clients(entries, a.distinct, seed=1, round_idx=3)
    for _, d in base:  # pageable host tensors, as unpickling produces them; touch every page once
        for t in d.values():
            t.add_(0)
    ns = sample_nums(a.K)
    nbytes = sum(t.numel() * t.element_size() for t in base[0][1].values())
    res = {"K": a.K, "bytes_per_client": nbytes}

    args = _Args()
    agg = MI355XServerAggregator(torch.nn.Linear(1, 1), args)
    agg.set_model_params = lambda p: None  # no torchvision here: the server model is a stand-in
    server = FedMLAggregator(None, None, 0, {}, {}, {}, a.K, dev, args, agg)
    rounds = []
    for r in range(3):
        per = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.K):
            d = OrderedDict(base[i % a.distinct][1])
            s = time.perf_counter()
            server.add_local_trained_result(i, d, ns[i])
            per.append(time.perf_counter() - s)
        t1 = time.perf_counter()
        server.check_whether_all_receive()
        averaged, _, _ = server.aggregate()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rounds.append({"arrival_ms_median": statistics.median(per) * 1e3,
                       "arrival_GBps": nbytes / statistics.median(per) / 1e9,
                       "all_arrivals_ms": (t1 - t0) * 1e3, "aggregate_ms": (t2 - t1) * 1e3})
    res["mi355x"] = rounds[-1]
    res["mi355x_all_rounds"] = rounds

    # the reference's flow on the same GPU
    raw = []
    per = []
    for i in range(a.K):
        d = OrderedDict(base[i % a.distinct][1])
        torch.cuda.synchronize()
        s = time.perf_counter()
        for k in d.keys():
            d[k] = d[k].to(dev)
        torch.cuda.synchronize()
        per.append(time.perf_counter() - s)
        raw.append((ns[i], d))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    _eager_fedavg(raw)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res["reference_flow_on_gpu"] = {"arrival_ms_median": statistics.median(per) * 1e3,
                                    "arrival_GBps": nbytes / statistics.median(per) / 1e9,
                                    "aggregate_ms": (t2 - t1) * 1e3}
    print(json.dumps(res, indent=1))
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/xsilo_bench.json", "w"), indent=1)


if __name__ == "__main__":
    main()
