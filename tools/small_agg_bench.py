"""FedMLAggOperator.agg at the small configs (1: 4 clients x LogisticRegression
MNIST; 2: 32 clients x CNN_WEB), where fixed per-call costs dominate: the
call on host dicts and on device dicts, against the reference's own loop
(agg_operator.py:35-44, restated inline) in torch eager on the CPU and on
the GPU.  Medians over many calls.

    python tools/small_agg_bench.py
"""
from __future__ import annotations

import copy
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import shapes  # noqa: E402
from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd.synth import host_clients  # noqa: E402


class _Args:
    federated_optimizer = "FedAvg"


def _eager(raw):
    training_num = 0
    for n, _ in raw:
        training_num += n
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


def _time(fn, make, reps, sync):
    ts = []
    for r in range(reps + 5):
        lst = make()
        if sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(lst)
        if sync:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        if r >= 5:
            ts.append((t1 - t0) * 1e6)
    return round(statistics.median(ts), 1)


def main():
    dev = torch.device("cuda:0")
    res = {}
    for cfg, model, K in (("cfg1", "lr_mnist", 4), ("cfg2", "cnn_web", 32)):
        raw = host_clients(shapes.MODELS[model](), K, seed=1)
        draw = [(n, OrderedDict((k, t.to(dev)) for k, t in d.items())) for n, d in raw]

        def host_list():
            return [(n, OrderedDict(d)) for n, d in raw]

        def dev_list():
            return [(n, OrderedDict(d)) for n, d in draw]

        args = _Args()
        r = {
            "agg_host_dicts_us": _time(lambda l: FedMLAggOperator.agg(args, l), host_list, 200, True),
            "agg_device_dicts_us": _time(lambda l: FedMLAggOperator.agg(args, l), dev_list, 200, True),
            "reference_loop_cpu_us": _time(_eager, host_list, 200, False),
            "reference_loop_gpu_eager_us": _time(_eager, dev_list, 200, True),
            "cpu_threads": torch.get_num_threads(),
        }
        res[cfg] = r
        print(cfg, r, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/small_agg_bench.json", "w"), indent=1)


if __name__ == "__main__":
    main()
