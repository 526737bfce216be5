"""End-to-end (host -> HBM -> host) aggregation rates at config 3 (tool).

    python tools/e2e_bench.py [--K 128] [--cpu-ref]

The north star's path starts and ends in host memory: client updates arrive
from the cross-silo transport as host state dicts and the averaged model is
broadcast back.  Measured here on 128 ResNet-50 clients (13.1 GB of host
inputs, pageable, one tensor per key as unpickling produces):

  ingest     ClientBucket.put per client at arrival (pinned staging + async
             H2D on a copy stream), GB/s over all clients
  round_end  after the last put: wait for ingest, reduce, D2H to independent
             host tensors — the latency the server adds once the last client
             is in
  agg_call   FedMLAggOperator.agg(args, host_list): the reference's call shape
             with everything inside one call (allocate rows, stage all
             clients, reduce, copy back)
  cpu_ref    the reference's own CPU loop on the same inputs (optional)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import shapes  # noqa: E402
from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd.bucket import ClientBucket  # noqa: E402
from fedml_amd.synth import sample_nums  # noqa: E402


def make_clients(entries, K, dev):
    """Host clients: per-key pageable tensors (generated on the GPU, copied down)."""
    n_f = shapes.numel(entries, torch.float32)
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(n_f, generator=g, device=dev) * 0.05
    ns = sample_nums(K)
    raw = []
    for i in range(K):
        flat = (base + 0.01 * torch.randn(n_f, generator=g, device=dev)).cpu()
        d = OrderedDict()
        off = 0
        for k, s, dt in entries:
            n = 1
            for x in s:
                n *= x
            if dt == torch.int64:
                d[k] = torch.full(s, 3 + i, dtype=torch.int64)
            else:
                d[k] = flat[off:off + n].view(s).clone()  # own storage per key, like unpickled tensors
                off += n
        raw.append((ns[i], d))
    return raw


def link_rates(dev, client):
    """Raw ceilings on this box: PCIe H2D/D2H from pinned and pageable host
    memory (1 GiB), and the native host pack of one client at 1/8/16 threads."""
    import ctypes

    from fedml_amd import _native as nat

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
        out[name] = 3 * nb / (time.perf_counter() - t0) / 1e9
    ts = list(client.values())
    n = len(ts)
    tot = sum(t.numel() * t.element_size() for t in ts)
    stage = torch.empty(tot // 4 + 64).pin_memory()
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += t.numel() * t.element_size()
    args = ((ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]), (ctypes.c_int64 * n)(*offs),
            (ctypes.c_int64 * n)(*[t.numel() * t.element_size() for t in ts]), n)
    for th in (1, 8, 16):
        nat.lib().fedagg_host_pack(stage.data_ptr(), *args, th)
        t0 = time.perf_counter()
        for _ in range(5):
            nat.lib().fedagg_host_pack(stage.data_ptr(), *args, th)
        out[f"host_pack_GBps_t{th}"] = 5 * tot / (time.perf_counter() - t0) / 1e9
    del pinned, pageable, d, stage
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--cpu-ref", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    entries = shapes.resnet50()
    raw = make_clients(entries, a.K, dev)
    in_bytes = sum(t.numel() * t.element_size() for _, d in raw for t in d.values())
    res = {"K": a.K, "host_input_bytes": in_bytes, "host_threads": torch.get_num_threads()}
    res.update(link_rates(dev, raw[0][1]))

    # ingest at arrival + round end
    bucket = ClientBucket(entries, a.K, dev)
    outs = bucket.new_outputs()
    for rep in range(2):  # rep 0 warms the pinned staging and the allocator
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        per_client = []
        for i, (n, d) in enumerate(raw):
            c0 = time.perf_counter()
            bucket.put(i, d, n)
            per_client.append(time.perf_counter() - c0)
        t1 = time.perf_counter()
        bucket.reduce_into(outs, bucket.weights([n for n, _ in raw]))
        host = bucket.to_host(outs)
        t2 = time.perf_counter()
    res["ingest_s"] = t1 - t0
    res["ingest_GBps"] = in_bytes / (t1 - t0) / 1e9
    res["ingest_per_client_ms_median"] = sorted(per_client)[len(per_client) // 2] * 1e3
    res["round_end_ms"] = (t2 - t1) * 1e3
    res["e2e_ingest_plus_round_end_s"] = t2 - t0
    assert list(host.keys()) == [e[0] for e in entries]

    # round-end breakdown (after every put has been issued)
    bd = {}
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    t0 = time.perf_counter()
    bucket.sync_ingest()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    bucket.reduce_into(outs, bucket.weights([n for n, _ in raw]))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host = bucket.to_host(outs)
    t3 = time.perf_counter()
    host2 = bucket.to_host(outs, into=host)  # into existing tensors (model.load_state_dict analogue)
    t4 = time.perf_counter()
    pinned_only = bucket._result_host[torch.float32]
    t5 = time.perf_counter()
    pinned_only.copy_(outs[torch.float32][:pinned_only.numel()])
    t6 = time.perf_counter()
    bd.update(drain_pending_h2d_ms=(t1 - t0) * 1e3, reduce_ms=(t2 - t1) * 1e3,
              to_host_fresh_tensors_ms=(t3 - t2) * 1e3, to_host_into_existing_ms=(t4 - t3) * 1e3,
              d2h_only_ms=(t6 - t5) * 1e3)
    assert all(host2[k] is host[k] for k in host)
    res["round_end_breakdown"] = bd

    # the pipelined round end (reduce_to_host: chunked reduce, D2H on a copy
    # stream, host scatter into pooled pre-touched tensors, all overlapped),
    # timed like round_end above: after every put, through the last byte on the host
    w = bucket.weights([n for n, _ in raw])
    pl = []
    for rep in range(4):  # rep 0 builds the chunk plan and the first pool
        for i, (n, d) in enumerate(raw):
            bucket.put(i, d, n)
        t1 = time.perf_counter()
        piped = bucket.reduce_to_host(w)
        pl.append((time.perf_counter() - t1) * 1e3)
        time.sleep(0.2)  # the next round's ingest time, in which the pool refills
    res["round_end_pipelined_ms"] = sorted(pl[1:])[len(pl[1:]) // 2]
    res["round_end_pipelined_ms_all"] = pl
    sweep = {}
    for ch in (4, 8, 16, 32):
        ts = []
        for rep in range(4):
            for i, (n, d) in enumerate(raw):
                bucket.put(i, d, n)
            t1 = time.perf_counter()
            bucket.reduce_to_host(w, chunks=ch)
            ts.append((time.perf_counter() - t1) * 1e3)
            time.sleep(0.2)
        sweep[ch] = sorted(ts[1:])[1]
    res["round_end_pipelined_chunk_sweep_ms"] = sweep
    res["pipelined_equals_serial"] = bool(all(torch.equal(piped[k], host[k]) for k in host))
    # A/B of the per-piece wait: the same pipelined round end with the range
    # reductions waiting for their own H2D pieces of the last clients ("piece")
    # or for every pending H2D first ("full", as before), interleaved
    ab = {"piece": [], "full": []}
    for rep in range(8):
        arm = "piece" if rep % 2 else "full"
        for i, (n, d) in enumerate(raw):
            bucket.put(i, d, n)
        if arm == "full":
            bucket._pending_other = True  # forces the whole-ingest wait
        t1 = time.perf_counter()
        bucket.reduce_to_host(w)
        ab[arm].append((time.perf_counter() - t1) * 1e3)
        time.sleep(0.2)
    res["round_end_piece_wait_ab_ms"] = {k: sorted(v)[len(v) // 2] for k, v in ab.items()}
    res["round_end_piece_wait_ab_all"] = ab

    # FAGG wire messages: ingest straight from the receive buffers
    from fedml_amd import wire

    msgs = [wire.encode(d, n) for n, d in raw]
    pinned_msgs = []
    for m in msgs[:32]:
        t = torch.empty(len(m), dtype=torch.uint8).pin_memory()
        t.numpy()[:] = memoryview(m)
        pinned_msgs.append(t)
    wb = {}
    for label, ms in (("pageable", msgs), ("pinned", [t.numpy() for t in pinned_msgs])):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, m in enumerate(ms):
                bucket.put_encoded(i, m)
            bucket.sync_ingest()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        wb[f"put_encoded_{label}_GBps"] = sum(len(m) for m in ms) / dt / 1e9
    t0 = time.perf_counter()
    _ = [wire.encode(d, n) for n, d in raw[:16]]
    wb["encode_GBps_client_side"] = sum(len(m) for m in msgs[:16]) / (time.perf_counter() - t0) / 1e9
    res["wire"] = wb

    # the reference's call shape
    args = type("Args", (), {"federated_optimizer": "FedAvg"})()
    times = []
    for rep in range(2):
        lst = [(raw[0][0], OrderedDict(raw[0][1]))] + raw[1:]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = FedMLAggOperator.agg(args, lst)
        times.append(time.perf_counter() - t0)
    res["agg_call_s"] = min(times)
    res["agg_call_GBps"] = in_bytes / min(times) / 1e9
    ok = all(torch.equal(out[k], host[k]) for k in host)
    res["agg_call_equals_bucket_path"] = bool(ok)

    if a.cpu_ref:
        from oracle import cpu_baseline as cb

        r = cb.time_fedavg(raw, reps=1)
        res["cpu_ref_s"] = r["median_s"]
        res["cpu_ref_threads"] = r["threads"]
        lst = [(raw[0][0], OrderedDict(raw[0][1]))] + raw[1:]
        ref = cb.fedavg(lst)
        res["gpu_equals_cpu_ref"] = bool(all(torch.equal(ref[k], host[k]) for k in host))
    print(json.dumps(res, indent=1), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/e2e.json", "w"), indent=1)


if __name__ == "__main__":
    main()
