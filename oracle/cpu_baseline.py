"""The reference's CPU FedAvg, restated in torch eager — TEST/BASELINE ONLY.

Only bench.py's cpu_baseline leg and tests/ use this.  It is the same per-key,
per-client loop as python/fedml/ml/aggregator/agg_operator.py:35-44 (and
simulation/sp/fedavg/fedavg_api.py:144-159): `avg[k] = p_0[k] * w` then
`avg[k] += p_i[k] * w` with w = n_i / Σn as a Python float, executed by
torch's CPU kernels — i.e. exactly the arithmetic and the dispatch pattern
FedML's server runs today.  tests/test_oracle_golden.py::test_cpu_baseline_is_reference
pins it bit for bit to the golden vectors.
"""
from __future__ import annotations

import os
import statistics
import time
from collections import OrderedDict
from typing import List, Tuple

import torch


def fedavg(raw_grad_list: List[Tuple[float, "OrderedDict[str, torch.Tensor]"]]) -> "OrderedDict[str, torch.Tensor]":
    training_num = 0
    for n, _ in raw_grad_list:
        training_num += n
    (num0, avg_params) = raw_grad_list[0]
    for k in avg_params.keys():
        for i in range(len(raw_grad_list)):
            n, params = raw_grad_list[i]
            w = n / training_num
            if i == 0:
                avg_params[k] = params[k] * w
            else:
                avg_params[k] += params[k] * w
    return avg_params


def time_fedavg(raw_grad_list, reps: int = 5, threads: int | None = None) -> dict:
    """Median wall time of fedavg over `reps` runs after one warm-up.  Client
    0's dict is rebuilt before each run because the loop rebinds its keys."""
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        c0 = OrderedDict(raw_grad_list[0][1])
        ts = []
        for r in range(reps + 1):
            lst = [(raw_grad_list[0][0], OrderedDict(c0))] + list(raw_grad_list[1:])
            t0 = time.perf_counter()
            fedavg(lst)
            dt = time.perf_counter() - t0
            if r:
                ts.append(dt)
        return {"median_s": statistics.median(ts), "min_s": min(ts), "threads": threads, "reps": reps}
    finally:
        torch.set_num_threads(old)
