"""FedMLAggOperator.agg on device-resident state dicts (FedML's `using_gpu`
server: every client tensor already moved to the GPU one by one,
ml_engine_adapter.py:234-254) at config 3: 128 clients x 320 ResNet-50 keys =
40,960 separate device tensors.  Reports wall time per agg() call (host side
included) next to the GPU time of the reduction launches.

    python tools/devdict_bench.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from fedml_amd import shapes  # noqa: E402
from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd.synth import sample_nums  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--chunks", default="", help="comma list overriding agg_operator._CHUNK_KEYS (e.g. 4,12,48)")
    ap.add_argument("--tail", type=int, default=0, help="override agg_operator._TAIL_CHUNK")
    ap.add_argument("--ab-weights", action="store_true",
                    help="also time agg() with the weights in the first table's H2D vs a separate upload, "
                         "interleaved (agg_operator._WEIGHTS_IN_TABLE)")
    a = ap.parse_args()
    if a.chunks:
        from fedml_amd import agg_operator as ao

        ao._CHUNK_KEYS = tuple(int(x) for x in a.chunks.split(","))
    if a.tail:
        from fedml_amd import agg_operator as ao

        ao._TAIL_CHUNK = a.tail
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    ents = shapes.resnet50()
    ns = sample_nums(a.K)
    raw = []
    for i in range(a.K):
        d = OrderedDict()
        for k, s, dt in ents:
            if dt == torch.int64:
                d[k] = torch.full(s, 3 + i, dtype=torch.int64, device=dev)
            else:
                d[k] = torch.randn(s, generator=g, device=dev) * 0.05
        raw.append((ns[i], d))
    args = type("Args", (), {"federated_optimizer": "FedAvg"})()
    c0 = OrderedDict(raw[0][1])
    times, gpu = [], []
    for r in range(a.reps + 1):
        lst = [(raw[0][0], OrderedDict(c0))] + raw[1:]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        FedMLAggOperator.agg(args, lst)
        e1.record()
        t1 = time.perf_counter()  # host returns (launches enqueued)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if r:
            times.append((t1 - t0, t2 - t0))
            gpu.append(e0.elapsed_time(e1))
    # host-side breakdown of the native-walker path (agg_operator._reduce_device_walked)
    import agg_breakdown  # noqa: F401  (tools/agg_breakdown.py)

    bd = agg_breakdown.breakdown([(raw[0][0], OrderedDict(c0))] + raw[1:], a.reps)
    res = {"K": a.K, "tensors": a.K * len(ents), "chunks": a.chunks or "default", "tail": a.tail or "default",
           "breakdown_ms": bd,
           "host_enqueue_ms_median": sorted(t[0] for t in times)[len(times) // 2] * 1e3,
           "wall_to_done_ms_median": sorted(t[1] for t in times)[len(times) // 2] * 1e3,
           "gpu_window_ms_median": sorted(gpu)[len(gpu) // 2]}
    if a.ab_weights:
        from fedml_amd import agg_operator as ao

        ab = {True: [], False: []}
        for r in range(4 * a.reps):
            flag = bool(r % 2)
            ao._WEIGHTS_IN_TABLE = flag
            lst = [(raw[0][0], OrderedDict(c0))] + raw[1:]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            FedMLAggOperator.agg(args, lst)
            torch.cuda.synchronize()
            ab[flag].append((time.perf_counter() - t0) * 1e3)
        ao._WEIGHTS_IN_TABLE = True
        res["ab_wall_to_done_ms"] = {"weights_in_table": sorted(ab[True])[len(ab[True]) // 2],
                                     "separate_upload": sorted(ab[False])[len(ab[False]) // 2]}
    print(json.dumps(res, indent=1))
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/devdict.json", "w"), indent=1)


if __name__ == "__main__":
    main()
