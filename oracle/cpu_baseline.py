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


def host_cpus() -> dict:
    """What this process may run on: os.cpu_count() (the machine), the
    affinity mask, the cgroup CPU quota, and the CPU model.  On the GPU box
    os.cpu_count() reports the whole machine while the job's share is
    smaller, so `usable` = min(affinity, quota) is the thread count a fair
    baseline uses."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    info["cgroup_quota_cpus"] = quota
    usable = info["affinity"]
    if quota is not None:
        usable = min(usable, max(1, int(quota + 0.5)))
    info["usable"] = usable
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["model"] = model
    return info


def time_fedavg(raw_grad_list, reps: int = 5, threads: int | None = None) -> dict:
    """Median wall time of fedavg over `reps` runs after one warm-up.  Client
    0's dict is rebuilt before each run because the loop rebinds its keys."""
    if threads is None:
        threads = host_cpus()["usable"]
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
