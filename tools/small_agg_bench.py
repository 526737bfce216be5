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


def _time(fn, make, reps, sync, sync_after=None):
    """sync: drain the device before the call; sync_after (default: sync):
    also inside the timed region after it (device results).  A host-dict
    agg() returns host tensors that already hold the result, like the
    reference loop, so it is timed without a trailing synchronize."""
    sync_after = sync if sync_after is None else sync_after
    ts = []
    for r in range(reps + 5):
        lst = make()
        if sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(lst)
        if sync_after:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        if r >= 5:
            ts.append((t1 - t0) * 1e6)
    return round(statistics.median(ts), 1)


def _one_thread(fn):
    old = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        return fn()
    finally:
        torch.set_num_threads(old)


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
        from fedml_amd import agg_operator as ao

        wk = ao._walker()
        keys = list(raw[0][1].keys())
        ws = [n / sum(n for n, _ in raw) for n, _ in raw]
        ao._reduce_host_round(wk, [d for _, d in raw], keys, ws)  # resolve the function pointers once
        ao._reduce_device_round(wk, [d for _, d in draw], keys, ws)
        r = {
            "native_host_round_us": _time(lambda l: wk.host_round([d for _, d in l], keys, ws, ao._HOST_ROUND_FN, 0,
                                                                  ao._HOST_ROUND_MAX_BYTES), host_list, 500, True,
                                          False),
            "agg_host_dicts_us": _time(lambda l: FedMLAggOperator.agg(args, l), host_list, 500, True, False),
            "agg_device_dicts_us": _time(lambda l: FedMLAggOperator.agg(args, l), dev_list, 500, True),
            # host time of the call alone (the result is stream-ordered, as every device path's)
            "agg_device_dicts_issue_us": _time(lambda l: FedMLAggOperator.agg(args, l), dev_list, 500, True, False),
            "native_device_round_us": _time(
                lambda l: wk.device_round([d for _, d in l], keys, ws, ao._DEVICE_ROUND_FN,
                                          torch._C._cuda_getCurrentRawStream), dev_list, 500, True),
            "reference_loop_cpu_us": _time(_eager, host_list, 500, False),
            "reference_loop_cpu_1thread_us": _one_thread(lambda: _time(_eager, host_list, 500, False)),
            "reference_loop_gpu_eager_us": _time(_eager, dev_list, 200, True),
            "cpu_threads": torch.get_num_threads(),
        }
        res[cfg] = r
        print(cfg, r, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/small_agg_bench.json"
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
