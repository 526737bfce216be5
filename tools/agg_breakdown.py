"""Host-side cost breakdown of FedMLAggOperator.agg on device-resident dicts
(tool only; used by tools/devdict_bench.py)."""
from __future__ import annotations

import statistics
import time

import torch

from fedml_amd import _native as nat
from fedml_amd import agg_operator as ao
from fedml_amd import kernels as kn


def breakdown(lst, reps: int = 5) -> dict:
    dicts = [d for _, d in lst]
    keys = list(dicts[0].keys())
    w = ao._walker()
    t = {"walk": [], "outputs": [], "plans": [], "launch": []}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev_idx, codes, numels, tables = w.walk(dicts, keys)
        t1 = time.perf_counter()
        dev = torch.device("cuda", dev_idx)
        outs = [torch.empty(dicts[0][k].shape, dtype=torch.float32 if c == nat.DT_I64 else dicts[0][k].dtype,
                            device=dev) for k, c in zip(keys, codes)]
        t2 = time.perf_counter()
        plans = {}
        for c in tables:
            ns = [o.numel() for o, cc in zip(outs, codes) if cc == c]
            plans[c] = (kn.MultiPlan(ns, ao._CODE_DT[c]), [o.data_ptr() for o, cc in zip(outs, codes) if cc == c])
        t3 = time.perf_counter()
        w32 = kn.upload_f32([1.0 / len(dicts)] * len(dicts), dev)
        for c, (plan, ops) in plans.items():
            plan.launch(tables[c], ops, w32, len(dicts), dev)
        t4 = time.perf_counter()
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            t[k].append(v * 1e3)
    torch.cuda.synchronize()
    return {k: round(statistics.median(v), 3) for k, v in t.items()}
