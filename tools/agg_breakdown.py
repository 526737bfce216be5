"""Host-side cost breakdown of FedMLAggOperator.agg on device-resident dicts
(tool only; used by tools/devdict_bench.py)."""
from __future__ import annotations

import statistics
import time

import torch

from fedml_amd import agg_operator as ao
from fedml_amd import kernels as kn


def breakdown(lst, reps: int = 5) -> dict:
    """Host time of the pipelined native-walker path, by phase, summed over
    its chunks (agg_operator._reduce_device_walked)."""
    dicts = [d for _, d in lst]
    keys = list(dicts[0].keys())
    K = len(dicts)
    w = ao._walker()
    t = {"order": [], "walk_alloc": [], "plans": [], "launch": [], "weights": [], "to_first_launch": []}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        order = w.order_by_size(dicts[0], keys)
        tw = tp = tl = 0.0
        t1 = time.perf_counter()
        w32 = None
        tu = first = 0.0
        for idx in ao._chunks(order):
            a = time.perf_counter()
            dev_idx, codes, numels, tables, outs, out_tables = w.walk(dicts, [keys[i] for i in idx], True)
            b = time.perf_counter()
            dev = torch.device("cuda", dev_idx)
            if w32 is None:
                u = time.perf_counter()
                w32 = kn.upload_f32([1.0 / K] * K, dev)
                tu = time.perf_counter() - u
            plans = {c: ao._multi_plan([n for n, cc in zip(numels, codes) if cc == c], c, 0) for c in tables}
            c_ = time.perf_counter()
            for c, plan in plans.items():
                plan.launch(tables[c], out_tables[c], w32, K, dev)
            d = time.perf_counter()
            if not first:
                first = d - t0
            tw, tp, tl = tw + (b - a), tp + (c_ - b), tl + (d - c_)
        for k, v in zip(t, (t1 - t0, tw, tp - tu, tl, tu, first)):
            t[k].append(v * 1e3)
    torch.cuda.synchronize()
    return {k: round(statistics.median(v), 3) for k, v in t.items()}
