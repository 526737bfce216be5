#!/usr/bin/env python
"""Headline benchmark: device-resident FedAvg aggregation on MI355X.

One step = one server aggregation round over client updates already resident
in HBM: host computes the weights w_i = n_i/Σn, and the weighted-sum kernels
reduce every client row (one launch per dtype group).

Default workload = BASELINE.json config 3: 128 clients x ResNet-50 state dict
(25,610,152 fp32 + 53 int64 elements per client), synthetic data generated
in HBM.

Every config keeps BASELINE.json's client count (4 / 32 / 128 / 512 / 64;
`plan_clients`).  With --gpus N (one process per GPU) the round keeps it too
(strong scaling, ``--clients-total``, default the config's K):

  --mode param (default)  every rank holds ITS KEYS of every client (whole
                          keys dealt to ranks by bytes, the same partition as
                          the in-process fedml_amd.multidev bucket) and
                          reduces them in the reference order: no exchange,
                          bit-exact with one GPU.  The same run then measures
                          the client axis below on the same clients and nests
                          it under "exchange" (north_star's RCCL
                          reduce-scatter over xGMI; --no-exchange skips it).
  --mode client           every rank holds its K/N clients' whole updates,
                          computes an fp32 partial and joins one chunked RCCL
                          reduce-scatter (timed separately on the comm stream).
  --weak                  round 2's weak scaling: every rank gets the
                          config's K clients of its own.

    python bench.py                       # 1 GPU, default steps
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8
    python bench.py --gpus 8              # the same: bench.py spawns the 8 ranks itself

In --mode param every multi-GPU line also nests "inprocess": rank 0 alone
drives all N GPUs from ONE process through fedml_amd.multidev.MultiDeviceBucket
(the only multi-GPU mode FedML's single server process can use), same clients,
per-device kernel GB/s and roofline fraction (--no-inprocess skips it).

Prints ONE JSON line on rank 0 (contract in the task statement); at N = 1 the
cpu_baseline leg times the reference's own CPU loop (oracle/cpu_baseline.py)
over the FULL workload (every key, every client) at the job's CPU quota and
at one thread.  `--op median` lines also carry roofline.valu: the median's
sorting networks are bound by VALU issue above ~128 clients, so the executed
VALU instructions of its kernel (profiles/median_valu.json, an SQ pass) at 4
cycles per wave64 instruction per SIMD are set against the kernel time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from fedml_amd import shapes  # noqa: E402
from fedml_amd.bucket import ClientBucket  # noqa: E402
from fedml_amd import multidev  # noqa: E402
from fedml_amd.layout import RowLayout  # noqa: E402
from fedml_amd.sharded import ClientAxisAggregator  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# packed fp32 vector peak (v_pk_fma_f32: 64 FLOP/clk/SIMD x 1,024 SIMDs x 2.4 GHz), the ceiling of
# the exact-difference Krum pair kernel, whose packed subtract + packed FMA are 3 flops per client pair and
# element (the centred-Gram kernel on the bf16 matrix cores is priced against HBM instead: it reads the
# rows once; MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_TFLOPS = 157.3
SIMDS = 256 * 4  # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4
VALU_HALF_RATE_CYCLES = 4  # min/max/med3/DPP wave64 issue cost per SIMD (profiles/r03/median_rsel/valu_rate_probe*.txt)
LSA_PRIME, LSA_QBITS = 2 ** 15 - 19, 10  # the reference's example LightSecAgg config (fedml_config.yaml:58-59)

CONFIGS = {
    "cfg1": dict(model="lr_mnist", K=4, desc="FedAvg 4 clients x LogisticRegression MNIST (7,850 params) fp32"),
    "cfg2": dict(model="cnn_web", K=32, desc="FedAvg 32 clients x LeNet CNN_WEB (62,006 params) fp32"),
    "cfg3": dict(model="resnet50", K=128,
                 desc="FedAvg 128 clients x ResNet-50 state dict (25,610,152 fp32 + 53 int64) fp32"),
    "cfg4": dict(model="vit_b16", K=512, desc="FedAvg 512 clients x ViT-B/16 (86,567,656) bf16"),
    "cfg5": dict(model="llama2_7b_lora", K=64, desc="FedAvg 64 clients x Llama-2-7B LoRA r=8 q/v fp32"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="param", choices=["client", "param"],
                    help="multi-GPU partitioning (ignored at 1 GPU): param = whole keys per rank, no exchange; "
                         "client = clients per rank + RCCL reduce-scatter")
    ap.add_argument("--clients-total", type=int, default=None,
                    help="multi-GPU: clients of the round over all ranks (default: the config's K)")
    ap.add_argument("--weak", action="store_true",
                    help="multi-GPU: every rank aggregates the config's K clients of its own (weak scaling)")
    ap.add_argument("--chunks", type=int, default=8, help="client mode: reduce-scatter pipeline depth")
    ap.add_argument("--acc", default="reference", choices=["reference", "fp32"],
                    help="bf16/f16 accumulation: torch's per-op chain (bit-exact) or fp32")
    ap.add_argument("--fedopt", nargs="?", const="sgd", default=None,
                    choices=["sgd", "adam", "adamw", "adagrad", "rmsprop"],
                    help="1 GPU: FedOpt server step fused into the reduction (config 5: SGD lr=1.0 momentum 0.9, "
                         "or Adam / Adagrad lr=1.0 with torch defaults)")
    ap.add_argument("--op", default="fedavg", choices=["fedavg", "median", "secagg", "lsa", "krum", "dist2", "clip",
                                                       "rlr", "mpi"],
                    help="1 GPU: the reduction measured (median = the wise_median defense kernel; secagg = "
                         "LightSecAgg's int64 sum mod p; lsa = its fused mask-cancel / de-quantize reconstruction; "
                         "krum / dist2 / clip = the distance defenses' kernels; rlr = the robust-learning-rate "
                         "defense's fused pass; mpi = the MPI simulation's fl(fl(p n_i) / N) order, "
                         "fedagg_wsum_muldiv)")
    ap.add_argument("--pair-distance", default="auto", choices=["auto", "gram", "exact"],
                    help="--op krum: the centred Gram on the bf16 matrix cores with an exact three-way split "
                         "(K <= 128) or the exact-difference VALU kernel")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = host-staged collectives, for rehearsing N ranks on one GPU (not a benchmark)")
    ap.add_argument("--clients", type=int, default=None,
                    help="1 GPU: clients per GPU instead of the config's (e.g. config 4's median over all 512 "
                         "clients: the median does not split along the client axis)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exchange", action="store_true",
                    help="multi-GPU --mode param: skip the nested client-axis (RCCL reduce-scatter) measurement")
    ap.add_argument("--cpu-reps", type=int, default=5, help="cpu_baseline: timed runs after one warm-up")
    ap.add_argument("--no-inprocess", action="store_true",
                    help="multi-GPU --mode param: skip the nested one-process measurement (MultiDeviceBucket over "
                         "the N GPUs, the mode FedML's single server process uses)")
    ap.add_argument("--spawn-probe", action="store_true", help=argparse.SUPPRESS)  # CPU test of the self-launch
    return ap.parse_args(argv)


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, probe: bool = False) -> int:
    """`python bench.py --gpus N` without torch.distributed.run: start N
    worker processes of this script, one per GPU, with torchrun's environment
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), wait for them and
    return the first failing exit code (0 if all succeed).  The parent never
    touches the GPU (no HIP call before or after the spawn: the workers start
    as fresh processes, not forks), and rank 0 prints the JSON line."""
    import signal
    import subprocess

    assert not torch.cuda.is_initialized(), "the launcher must not initialise HIP"
    port = free_port()
    procs = []

    def stop_all():
        for q in procs:
            if q.poll() is None:
                q.terminate()

    def on_signal(signum, frame):  # the launcher is stopped (a time limit): take the ranks with it
        stop_all()
        raise SystemExit(128 + signum)

    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    stop_all()  # a rank died: the others would wait in a collective forever
            time.sleep(0.05)
    finally:
        stop_all()
        for p in procs:
            p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    if probe:
        print(json.dumps({"probe": "parent", "cuda_initialized": torch.cuda.is_initialized(),
                          "exit_codes": [p.returncode for p in procs]}), flush=True)
    return rc


def plan_clients(config: str, world: int, rank: int, mode: str, clients_total=None, weak: bool = False,
                 clients=None):
    """(K_total, K_loc, first): the round's clients over all ranks, this
    rank's count and the index of its first client.  mode is "single" at one
    GPU, else "param" (every rank holds its keys of ALL clients) or "client"
    (clients dealt to ranks, the first K_total % world ranks one more)."""
    K = CONFIGS[config]["K"]
    if clients is not None:
        if world > 1 or clients < 1:
            raise SystemExit("--clients is a 1-GPU override (>= 1)")
        K = clients
    weak = weak and world > 1
    if world > 1 and not weak:
        K_total = clients_total if clients_total is not None else K
        if K_total < 1:
            raise SystemExit("--clients-total must be >= 1")
    else:
        K_total = K * world
    if mode == "client" and not weak:
        base_k, extra = divmod(K_total, world)
        K_loc = base_k + (1 if rank < extra else 0)
        first = rank * base_k + min(rank, extra)
    elif mode == "client" or weak:
        K_loc, first = K, rank * K
    else:
        K_loc, first = K_total, 0
    if K_loc < 1:
        raise SystemExit(f"rank {rank} would hold no clients: --clients-total {K_total} < --gpus {world}")
    return K_total, K_loc, first


def fill_rows(rows: torch.Tensor, length: int, seed: int, round_idx: int = 0) -> None:
    """Synthetic updates in HBM: base ~ N(0, 0.05²), client_i = base + 0.01·ε_i
    (SURVEY.md §8(d)); int64 rows get round_idx + i."""
    K = rows.shape[0]
    if rows.dtype == torch.int64:
        for i in range(K):
            rows[i].fill_(round_idx + i)
        return
    g = torch.Generator(device=rows.device).manual_seed(seed)
    base = torch.randn(length, generator=g, device=rows.device) * 0.05
    eps = torch.empty(length, device=rows.device)
    for i in range(K):
        eps.normal_(0.0, 1.0, generator=g)
        rows[i, :length].copy_(base + 0.01 * eps)
        rows[i, length:].zero_()
    del base, eps


CPU_SAMPLE_BYTES = 13_400_000_000  # cpu_baseline: client bytes copied to the host (config 3 = 13.2 GB, all of it)


def host_round(bucket, clients=None) -> list:
    """The bench's round as the reference's CPU server holds it: K pageable
    per-key host tensors per client (contiguous slices of one host copy of
    each client's row; integer keys as int64 tensors), copied from HBM.
    clients: the first this many slots (default all)."""
    from collections import OrderedDict

    raw = []
    for i in range(bucket.capacity if clients is None else clients):
        d = OrderedDict()
        rows = {dt: g.rows[i, :g.length].cpu() for dt, g in bucket.groups.items()}
        for key, shape, dt in bucket.entries:
            g, j = bucket.where[key]
            t = rows[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].view(shape)
            d[key] = t.to(dt) if key in bucket.int_keys else t
        raw.append((bucket.sample_nums[i] if bucket.sample_nums[i] is not None else 1, d))
    return raw


def cpu_baseline(bucket, ns, reps: int) -> dict:
    """The reference's own CPU loop (agg_operator.py:35-44 in torch eager,
    oracle/cpu_baseline.py) on every key of the state dict and the same values
    as the HBM rows: all K clients while they fit CPU_SAMPLE_BYTES (config 3:
    the FULL workload), else the first K' clients that do (config 4's 512 x
    173 MB: a bounded sample; the unit is a rate, client-params/s).  Median of
    `reps` runs after one warm-up, at every CPU this job may use and at one
    thread."""
    from oracle import cpu_baseline as cb

    row_bytes = sum(g.length * g.rows.element_size() for g in bucket.groups.values())
    k_all = bucket.capacity
    k_s = max(1, min(k_all, CPU_SAMPLE_BYTES // max(1, row_bytes)))
    raw = host_round(bucket, k_s)
    raw = [(n, d) for n, (_, d) in zip(ns, raw)]
    cpus = cb.host_cpus()
    full = cb.time_fedavg(raw, reps=reps, threads=cpus["usable"])
    one = cb.time_fedavg(raw, reps=reps, threads=1)
    K = len(raw)
    n_elems = bucket.num_elements()
    del raw
    return {"value": K * n_elems / full["median_s"], "unit": "client-params/s", "cores": full["threads"],
            "kind": "port",
            "sample": ("full workload" if K == k_all else f"bounded sample: the first {K} of {k_all} clients") +
                      f": all {len(bucket.entries)} state-dict keys x {K} clients "
                      f"({n_elems:,} elements/client), torch-eager restatement of agg_operator.py:35-44, "
                      f"median of {reps} after 1 warm-up: {full['median_s'] * 1e3:.1f} ms/aggregation at "
                      f"{full['threads']} threads, {one['median_s'] * 1e3:.1f} ms at 1 thread",
            "threads": full["threads"],
            "cores_basis": "threads used = the CPUs this job may use (the box's cgroup quota), not the host's "
                           "nproc; see host",
            "ms_per_aggregation": round(full["median_s"] * 1e3, 2),
            "single_thread": {"value": K * n_elems / one["median_s"], "threads": 1,
                              "ms_per_aggregation": round(one["median_s"] * 1e3, 2)},
            "host": {"cpu_model": cpus["model"], "nproc": cpus["nproc"], "affinity_cpus": cpus["affinity"],
                     "cgroup_quota_cpus": cpus["cgroup_quota_cpus"]}}


def median_kernel_name(K: int, dt) -> str:
    """The kernel fedagg_median dispatches for K clients of aligned rows
    (median_dispatch in csrc/median.hip)."""
    name = str(dt).replace("torch.", "")
    packed = dt in (torch.bfloat16, torch.float16)
    if K <= 128:
        kmax = next(m for m in ((32, 64, 96, 128) if packed else (8, 16, 24, 32, 48, 64, 96, 128)) if K <= m)
        return f"median_{'pk16_' if packed else ''}kernel<{kmax}> ({name})"
    if K > 4096 or (not packed and 2048 < K <= 2560):
        return f"median_radix_stream_kernel ({name})"
    p, r = (4, 64) if K <= 256 else (4, 128) if K <= 512 else (8, 128) if K <= 1024 else \
        (16, 128) if K <= 2048 else (32, 128)
    return f"median_{'pk16_' if packed else ''}lanes_kernel<{p}, {r}> ({name})"


def table_key(config: str, mode: str, world: int, variant: str, clients: int) -> str:
    """Key of a measurement table entry: config, partitioning, variant and the
    clients per GPU it was measured at, e.g. "cfg4:single@K512",
    "cfg3:single:median@K128"."""
    return f"{config}:{mode if world > 1 else 'single'}" + (f":{variant}" if variant else "") + f"@K{clients}"


def load_traffic(config: str, mode: str, world: int, variant: str = "", clients: int = 128):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None.
    variant: "" for FedAvg, else the fused server step or the robust op."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = table_key(config, mode, world, variant, clients)
    try:
        return json.load(open(path)).get(key, {}).get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_median_valu(config: str, mode: str, world: int, variant: str, clients: int):
    """Executed VALU instructions per wave and waves per launch of the median
    kernel at this shape, from the committed SQ pass (profiles/median_valu.json,
    tools/median_valu.py), or None."""
    path = os.path.join(ROOT, "profiles", "median_valu.json")
    key = table_key(config, mode, world, variant, clients)
    try:
        return json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None


def client_axis_step(bucket, dom_dt, w_local, chunks: int, world: int):
    """The client-axis step over this rank's bucket: per dtype group the fp32
    partial of its clients (global weights) and the chunked reduce-scatter,
    16-bit models rounded once after the exchange.  Returns (step, launches
    per step of the dominant group, its algorithmic bytes, xGMI bytes per rank)."""
    aggs = {dt: ClientAxisAggregator(g.rows, g.length, chunks=chunks if dt == dom_dt else 1)
            for dt, g in bucket.groups.items()}

    def step(ev=None, cev=None):
        for dt, agg in aggs.items():
            agg.aggregate(w_local, events=ev if dt == dom_dt else None,
                          comm_events=cev if dt == dom_dt else None)
            if dt in (torch.bfloat16, torch.float16):
                agg.shard_in_model_dtype()  # the one rounding of a 16-bit model, after the exchange

    gd = bucket.groups[dom_dt]
    dom_bytes = gd.rows.shape[0] * gd.length * gd.rows.element_size() + gd.length * 4  # rows in, fp32 partial out
    xgmi_bytes = (world - 1) * aggs[dom_dt].piece * len(aggs[dom_dt].bounds) * 4
    return step, len(aggs[dom_dt].bounds), dom_bytes, xgmi_bytes


def run_timed(step, n_launch: int, steps: int, warmup: int, world: int, per_chunk: bool, timed_comm: bool):
    """W untimed steps, then K timed steps between barrier + synchronize on
    both sides.  Returns (elapsed s, MAX over ranks; kernel ms per step from
    the HIP events on the launch stream; comm-stream ms per step or None)."""
    def new_events(n):
        return [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(n)]

    for _ in range(warmup):
        step()
    evs = [new_events(n_launch) for _ in range(steps)]
    cevs = [new_events(n_launch) for _ in range(steps)] if timed_comm else [None] * steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        # the client-axis steps take one (start, end) pair per chunk; the rest one pair
        step(evs[s] if per_chunk else evs[s][0], cevs[s])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=torch.cuda.current_device(), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = sum(e0.elapsed_time(e1) for ev in evs for e0, e1 in ev) / steps  # per step
    comm_ms = sum(e0.elapsed_time(e1) for ev in cevs for e0, e1 in ev) / steps if timed_comm else None
    return elapsed, kern_ms, comm_ms


def reduce_rates(achieved: float, hbm_all: float, comm_ms, world: int, dev):
    """Over ranks: the slowest rank's kernel rate, the sum of the ranks' HBM
    rates and the mean comm-stream time."""
    t = torch.tensor([achieved], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)  # slowest rank's kernel
    achieved = float(t.item())
    t = torch.tensor([hbm_all, comm_ms or 0.0], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    hbm_all = float(t[0].item())
    if comm_ms is not None:
        comm_ms = float(t[1].item()) / world
    return achieved, hbm_all, comm_ms


def measure_client_axis(a, entries, n_elems: int, K_total: int, world: int, rank: int, dev) -> dict:
    """north_star's client-axis mode on the same round (the same K_total
    clients and sample counts): this rank's K_total/world clients' whole
    updates, the fp32 partial and the chunked RCCL reduce-scatter over xGMI.
    Runs after the headline in the same processes; returns the "exchange"
    object of the JSON line."""
    from fedml_amd.synth import sample_nums

    if K_total < world:
        return {"mode": "client", "skipped": f"{K_total} clients cannot cover {world} ranks on the client axis"}
    _, K_c, first_c = plan_clients(a.config, world, rank, "client", K_total)
    ns_all = sample_nums(K_total, seed=1)
    total_n = sum(ns_all)
    w = [n / total_n for n in ns_all[first_c:first_c + K_c]]
    bucket = ClientBucket(entries, K_c, dev, low_precision_acc=a.acc)
    for gi, (dt, g) in enumerate(bucket.groups.items()):
        fill_rows(g.rows, g.length, seed=1000 * rank + gi, round_idx=3)
    torch.cuda.synchronize()
    dom_dt = max(bucket.groups.items(), key=lambda kv: kv[1].length * kv[1].rows.element_size())[0]
    step, n_launch, dom_bytes, xgmi_bytes = client_axis_step(bucket, dom_dt, w, a.chunks, world)
    backend = dist.get_backend()
    timed_comm = backend == "nccl"
    elapsed, kern_ms, comm_ms = run_timed(step, n_launch, a.steps, a.warmup, world, True, timed_comm)
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9
    hbm_all = dom_bytes / (elapsed / a.steps) / 1e9
    achieved, hbm_all, comm_ms = reduce_rates(achieved, hbm_all, comm_ms, world, dev)
    ms = elapsed / a.steps * 1e3
    out = {"mode": "client", "backend": backend, "world_size": world,
           "collective": "reduce_scatter_tensor (RCCL over xGMI)" if backend == "nccl" else
           "reduce_scatter_tensor (gloo, host-staged: a rehearsal, not a measurement)",
           "clients_total": K_total, "clients_per_gpu": K_c, "chunks": n_launch,
           "value": K_total * n_elems / (elapsed / a.steps), "unit": "client-params/s",
           "ms_per_step": ms, "kernel_ms_per_step": round(kern_ms, 4),
           "kernel_gbps_slowest_rank": round(achieved, 1), "aggregate_gbps": round(hbm_all, 1),
           "xgmi_bytes_per_rank_per_step": xgmi_bytes,
           "comm_ms_per_step": round(comm_ms, 4) if comm_ms is not None else None,
           "parity": "fp32 partials summed across GPUs: |d| <= 2(K + log2 G + 1) 2^-24 sum|w_i p_i| vs one GPU "
                     "(ClientAxisAggregator.tolerance; tests/test_sharded_gloo.py)",
           "note": "same clients as the headline; comm_ms: mean over ranks of the chunks' reduce-scatter time on "
                   "the comm stream (overlapping the next chunk's reduction)"}
    del step, bucket
    torch.cuda.empty_cache()
    return out


def host_barrier(tag: str, world: int) -> None:
    """A barrier on the host only, through the rendezvous TCP store: around
    the one-process measurement an RCCL barrier would leave a spinning kernel
    on every waiting rank's GPU while rank 0 reduces there."""
    store = dist.distributed_c10d._get_default_store()
    store.add(tag, 1)
    while store.add(tag, 0) < world:
        time.sleep(0.005)


def measure_inprocess(a, entries, n_elems: int, K_total: int, world: int) -> dict:
    """The multi-GPU mode FedML's server can use: ONE process (the server is
    one process, python/fedml/__init__.py:330-348) driving `world` GPUs
    through fedml_amd.multidev.MultiDeviceBucket: whole keys per device, every
    device reducing its keys of all K_total clients in the reference order (no
    exchange, bit-exact with one GPU; cross_silo/server/fedml_aggregator.py:
    58-67 feeds it).  Device-resident rows, the same clients and weights as
    the headline; runs on rank 0 while the other ranks wait at a barrier with
    their rows freed (host_barrier).  Returns the "inprocess" object of the
    JSON line."""
    from fedml_amd.synth import sample_nums

    n_dev = torch.cuda.device_count()
    devices = [torch.device("cuda", i % n_dev) for i in range(world)]
    mb = multidev.MultiDeviceBucket(entries, K_total, devices, low_precision_acc=a.acc)
    for s, b in enumerate(mb.shards):
        with torch.cuda.device(b.device):
            for gi, (dt, g) in enumerate(b.groups.items()):
                fill_rows(g.rows, g.length, seed=5000 + 100 * s + gi, round_idx=3)
    ns = sample_nums(K_total, seed=1)
    w = mb.weights(ns)
    outs = [b.new_outputs() for b in mb.shards]
    doms = [b.dominant_dtype() for b in mb.shards]
    used = sorted({d.index for d in mb.devices})

    def sync_all():
        for i in used:
            torch.cuda.synchronize(i)

    def step(evs=None):
        for s, b in enumerate(mb.shards):  # every device's launches queued before any is waited for
            b.reduce_into(outs[s], w, events={doms[s]: evs[s]} if evs is not None else None)

    for _ in range(a.warmup):
        step()
    evs = []
    for _ in range(a.steps):
        per = []
        for b in mb.shards:
            with torch.cuda.device(b.device):
                per.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        evs.append(per)
    sync_all()
    t0 = time.perf_counter()
    for s in range(a.steps):
        step(evs[s])
    sync_all()
    elapsed = time.perf_counter() - t0
    per_dev = []
    total_bytes = 0
    for s, b in enumerate(mb.shards):
        g = b.groups[doms[s]]
        dom_bytes = K_total * g.length * g.rows.element_size() + \
            g.length * torch.empty((), dtype=g.out_dtype).element_size()
        kern_ms = sum(ev[s][0].elapsed_time(ev[s][1]) for ev in evs) / a.steps
        gbps = dom_bytes / (kern_ms / 1e3) / 1e9
        total_bytes += b.algorithmic_bytes()
        per_dev.append({"device": str(b.device), "keys": len(b.entries), "alg_bytes_per_step": dom_bytes,
                        "kernel_ms_per_step": round(kern_ms, 4), "gbps": round(gbps, 1),
                        "frac": round(gbps / HBM_PEAK_GBPS, 4)})
    ms = elapsed / a.steps * 1e3
    shared = len(used) < len(mb.shards)
    out = {"mode": "one process, G GPUs (fedml_amd.multidev.MultiDeviceBucket)", "devices": len(mb.shards),
           "distinct_gpus": len(used), "clients_total": K_total,
           "value": K_total * n_elems / (elapsed / a.steps), "unit": "client-params/s", "ms_per_step": ms,
           "slowest_device_kernel_ms": max(d["kernel_ms_per_step"] for d in per_dev),
           "per_device": per_dev, "aggregate_gbps": round(total_bytes / (elapsed / a.steps) / 1e9, 1),
           "aggregate_frac_of_n_peaks": round(total_bytes / (elapsed / a.steps) / 1e9 / (len(used) * HBM_PEAK_GBPS),
                                              4),
           "shard_balance": round(max(mb.shard_bytes()) / (sum(mb.shard_bytes()) / len(mb.shards)), 4),
           "parity": "bit-exact with one GPU (whole keys per device, reference client order; "
                     "tests/test_gpu_multidev.py)",
           "note": ("shards share one GPU here: a rehearsal of the launch pattern, not a multi-GPU rate"
                    if shared else "device-resident rows; reduce_to_host (D2H) excluded, as in the headline")}
    del mb, outs
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched as `python bench.py --gpus N`: become torchrun ourselves
        raise SystemExit(spawn_ranks(a.gpus, sys.argv[1:], probe=a.spawn_probe))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus > 1 and world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one process per GPU (or drop WORLD_SIZE "
                         "and let bench.py spawn them)")
    if a.spawn_probe:
        print(json.dumps({"probe": "rank", "rank": rank, "local_rank": local, "world": world,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}",
                          "cuda_initialized": torch.cuda.is_initialized()}), flush=True)
        return
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    cfg = CONFIGS[a.config]
    entries = shapes.MODELS[cfg["model"]]()
    full_layout = RowLayout(entries)
    n_elems = sum(sum(g.numels) for g in full_layout.groups.values())  # per client, the whole model
    mode = a.mode if world > 1 else "single"
    weak = a.weak and world > 1
    # this rank's clients: all of them (single / param axis) or its share (client axis)
    K_total, K_loc, first = plan_clients(a.config, world, rank, mode, a.clients_total, a.weak, a.clients)
    K = K_loc
    # the keys this rank reduces: all of them, or its whole-key shard (param axis)
    my_entries = entries
    if mode == "param":
        plan = multidev.shard_plan(entries, world)
        if len(plan) < world:
            raise SystemExit(f"{a.config} has data in {len(plan)} keys: too few for {world} ranks in --mode param")
        my_entries = plan[rank]

    from fedml_amd.synth import sample_nums
    ns_all = sample_nums(K_total, seed=1)
    ns_local = ns_all[first:first + K_loc]
    total_n = sum(ns_all)
    w_local = [n / total_n for n in ns_local]  # global weights of this rank's clients

    server = None
    sharded_opt = None
    if a.fedopt and mode == "client":
        bucket = ClientBucket(entries, K_loc, dev)  # integer buffers promoted into the fp32 row
        if set(bucket.groups) != {torch.float32}:
            raise SystemExit("--fedopt over several GPUs takes an fp32 model (integer buffers promoted)")
    elif a.fedopt:
        from collections import OrderedDict

        from fedml_amd.fedopt import FedOptServer

        init = OrderedDict((k, torch.zeros(s, dtype=d)) for k, s, d in my_entries)
        mine = {k for k, _, _ in my_entries}
        params = [p for p in shapes.param_names(entries) if p in mine]
        server = FedOptServer(init, params, K_loc, a.fedopt, 1.0, 0.9 if a.fedopt == "sgd" else 0.0, dev)
        bucket = server.bucket
    elif a.op in ("secagg", "lsa"):
        if world > 1:
            raise SystemExit("--op secagg / lsa is a 1-GPU measurement")
        # the model's elements as finite-field int64 rows (LightSecAgg's
        # transform_tensor_to_finite output), one group
        bucket = ClientBucket([(k, s, torch.int64) for k, s, _ in entries], K, dev, promote_ints=False)
    else:
        bucket = ClientBucket(my_entries, K_loc, dev, low_precision_acc=a.acc)
    for gi, (dt, g) in enumerate(bucket.groups.items()):
        if a.op in ("secagg", "lsa"):
            gen = torch.Generator(device=dev).manual_seed(1000 * rank + gi)
            g.rows.random_(0, LSA_PRIME, generator=gen)
        else:
            fill_rows(g.rows, g.length, seed=1000 * rank + gi, round_idx=3)
    torch.cuda.synchronize()

    groups = list(bucket.groups.items())
    dom_dt = max(groups, key=lambda kv: kv[1].length * kv[1].rows.element_size())[0]
    xgmi_bytes = 0

    # per-step work -------------------------------------------------------------
    if a.fedopt and mode == "client":
        from fedml_amd.sharded import ShardedFedOpt, buffer_ranges

        gd = bucket.groups[torch.float32]
        init = torch.zeros(gd.length, dtype=torch.float32, device=dev)
        sharded_opt = ShardedFedOpt(gd.rows, gd.length, init, a.fedopt, 1.0, 0.9 if a.fedopt == "sgd" else 0.0,
                                    chunks=a.chunks, buffers=buffer_ranges(bucket, shapes.param_names(entries)))

        def step(ev=None, cev=None):
            sharded_opt.aggregate(w_local, events=ev, comm_events=cev)

        n_launch = len(sharded_opt.agg.bounds)
        sharded_opt.aggregate(w_local)  # first step (no state read) before timing
        dom_bytes = K_loc * gd.length * 4 + gd.length * 4  # rows in, fp32 partial out (the step is 1/G of a pass)
        xgmi_bytes = (world - 1) * sharded_opt.agg.piece * len(sharded_opt.agg.bounds) * 4
    elif server is not None:
        for i, n in enumerate(ns_local):
            server.sample_num_dict[i] = n

        def step(ev=None, cev=None):
            server.aggregate(events=ev)

        n_launch = 1
        server.aggregate()  # first step (no momentum read) happens before timing
        dom_bytes = server.algorithmic_bytes()
    elif a.op == "median":
        from fedml_amd import defense as dfn

        if world > 1:
            raise SystemExit("--op median is a 1-GPU measurement")
        gd = bucket.groups[dom_dt]
        med_out = torch.empty(gd.padded, dtype=gd.rows.dtype, device=dev)  # the median is one of the inputs

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            dfn.median_rows(gd.d_ptrs, K, gd.length, med_out, aligned=True)
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = (K + 1) * gd.length * gd.rows.element_size()
    elif a.op == "rlr":
        # the robust-learning-rate defense: FedAvg chain + per-coordinate sign
        # sum + the lr rule, one pass over the fp32 row (threshold K/4)
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op rlr is a 1-GPU measurement")
        gd = bucket.groups[torch.float32]
        rlr_out = torch.empty(gd.padded, dtype=torch.float32, device=dev)
        rlr_w = kn.weights_for([n / sum(ns_local) for n in ns_local], torch.float32, dev)

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            kn.wsum_rlr_ptrs(gd.d_ptrs, rlr_w, K, gd.length, float(max(1, K // 4)), rlr_out, True)
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = (K + 1) * gd.length * 4
    elif a.op == "mpi":
        # the MPI simulation's term order (FedAVGAggregator.py:99-116) over the
        # dominant row: two roundings and a correctly rounded division per term
        from fedml_amd import _native as nat
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op mpi is a 1-GPU measurement")
        gd = bucket.groups[dom_dt]
        mpi_out = torch.empty(gd.padded, dtype=gd.out_dtype, device=dev)
        mpi_w = kn.muldiv_weights(dom_dt, [(n, sum(ns_local)) for n in ns_local], dev)
        code = kn._DT_CODE[dom_dt]
        call = lambda: nat.lib().fedagg_wsum_muldiv(  # noqa: E731
            code, gd.d_ptrs.data_ptr(), mpi_w.data_ptr(), K, gd.length, mpi_out.data_ptr(), nat.FEDAGG_ALIGNED16,
            nat.stream_handle())

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), "mpi")
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = K * gd.length * gd.rows.element_size() + gd.length * torch.empty((), dtype=gd.out_dtype).element_size()
    elif a.op in ("krum", "dist2", "clip"):
        # the distance defenses' kernels over the fp32 row's weight keys
        # (csrc/robust.hip): krum = the K x K pair kernel, dist2 = every
        # client's distance to a global row, clip = the clipped rebuild
        from fedml_amd import _native as nat
        from fedml_amd import defense as dfn
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op krum / dist2 / clip is a 1-GPU measurement")
        gd = bucket.groups[torch.float32]
        ref_row = gd.rows[K - 1].clone()  # a "global model" row
        if a.op == "krum":
            chunks, n_chunks = dfn.weight_chunks(gd, nat.PAIR_CHUNK, dev)
            pd_out = torch.empty((K, K), dtype=torch.float64, device=dev)
            gram = a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= dfn.GRAM_MAX_CLIENTS)
            work = dfn._work(nat.WORK_PAIRGRAM if gram else nat.WORK_PAIRDIST2, K, n_chunks, dev)
            pair_fn = nat.lib().fedagg_pairgram2_f32 if gram else nat.lib().fedagg_pairdist2_f32
            call = lambda: pair_fn(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, chunks.data_ptr(), n_chunks, pd_out.data_ptr(), work.data_ptr(),
                work.numel(), nat.stream_handle())
        elif a.op == "dist2":
            chunks, n_chunks = dfn.weight_chunks(gd, nat.DIST_CHUNK, dev)
            d_out = torch.empty(K, dtype=torch.float64, device=dev)
            work = dfn._work(nat.WORK_DIST2, K, n_chunks, dev)
            call = lambda: nat.lib().fedagg_dist2_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, ref_row.data_ptr(), chunks.data_ptr(), n_chunks, d_out.data_ptr(),
                work.data_ptr(), work.numel(), nat.stream_handle())
        else:
            clip_out = torch.empty_like(gd.rows)
            d_dst = kn.upload_i64([clip_out[i].data_ptr() for i in range(K)], dev)
            d_div = kn.upload_f32([1.0 + 0.01 * i for i in range(K)], dev)
            call = lambda: nat.lib().fedagg_clip_diff_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, ref_row.data_ptr(), d_div.data_ptr(), gd.length, d_dst.data_ptr(),
                nat.stream_handle())
        n_weight = sum(n for k, n in zip(gd.keys, gd.numels) if dfn.is_weight_param(k))
        gram = a.op == "krum" and (a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= 128))
        # krum, exact kernel: 3 flops (sub, mul, add) per client pair and weight element (VALU-bound);
        # krum, centred Gram on the bf16 matrix cores: the K weight rows read once (HBM-bound: its
        # six bf16 MFMAs per 32 columns need ~2/3 of the time the rows take to stream);
        # dist2: K rows + the reference row read once; clip: K rows in + K out + the reference row
        dom_bytes = {"krum": K * n_weight * 4 if a.op == "krum" and gram else 3 * K * (K - 1) // 2 * n_weight,
                     "dist2": (K + 1) * n_weight * 4, "clip": (2 * K + 1) * gd.length * 4}[a.op]
        krum_pair_flops = 2 * K * (K - 1) // 2 * n_weight  # one multiply-add per client pair and element

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), a.op)
            if ev is not None:
                ev[1].record()

        n_launch = 1
    elif a.op in ("secagg", "lsa"):
        from fedml_amd import _native as nat

        gd = bucket.groups[torch.int64]
        if a.op == "secagg":
            sec_out = torch.empty(gd.padded, dtype=torch.int64, device=dev)
            call = lambda: nat.lib().fedagg_sum_mod_i64(gd.d_ptrs.data_ptr(), K, gd.length, LSA_PRIME,  # noqa: E731
                                                        sec_out.data_ptr(), nat.FEDAGG_ALIGNED16, nat.stream_handle())
            dom_bytes = (K + 1) * gd.length * 8
        else:
            mask = torch.empty(gd.padded, dtype=torch.int64, device=dev).random_(0, LSA_PRIME)
            sec_out = torch.empty(gd.padded, dtype=torch.float32, device=dev)
            call = lambda: nat.lib().fedagg_lsa_reconstruct_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, gd.length, mask.data_ptr(), LSA_PRIME, LSA_QBITS, 1.0 / K,
                sec_out.data_ptr(), nat.FEDAGG_ALIGNED16, nat.stream_handle())
            dom_bytes = (K + 1) * gd.length * 8 + gd.length * 4

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), a.op)
            if ev is not None:
                ev[1].record()

        n_launch = 1
    elif mode in ("single", "param"):
        # one GPU, or this rank's whole-key shard of every client: the
        # single-GPU reduction over the bucket, no exchange
        outs = bucket.new_outputs()
        w = w_local if mode == "param" else bucket.weights(ns_local)

        def step(ev=None, cev=None):
            bucket.reduce_into(outs, w, events={dom_dt: ev} if ev is not None else None)

        n_launch = 1
        gd = bucket.groups[dom_dt]
        dom_bytes = K_loc * gd.length * gd.rows.element_size() + \
            gd.length * torch.empty((), dtype=gd.out_dtype).element_size()
    else:  # client axis: this rank's clients' partial + chunked RCCL reduce-scatter
        step, n_launch, dom_bytes, xgmi_bytes = client_axis_step(bucket, dom_dt, w_local, a.chunks, world)

    timed_comm = mode == "client" and world > 1 and a.backend == "nccl"
    elapsed, kern_ms, comm_ms = run_timed(step, n_launch, a.steps, a.warmup, world, mode == "client", timed_comm)
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9  # GB/s (GFLOP/s for the exact-difference krum kernel)
    hbm_all = dom_bytes / (elapsed / a.steps) / 1e9  # this rank's algorithmic bytes over the step time
    if world > 1:
        achieved, hbm_all, comm_ms = reduce_rates(achieved, hbm_all, comm_ms, world, dev)

    ms_per_step = elapsed / a.steps * 1e3
    gram_op = a.op == "krum" and (a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= 128))
    value = K_total * n_elems / (elapsed / a.steps)
    variant = a.fedopt or ("" if a.op == "fedavg" else a.op)
    if a.acc == "fp32" and dom_dt in (torch.bfloat16, torch.float16) and a.op == "fedavg":
        variant = (variant + "+" if variant else "") + "acc32"  # the fp32-accumulate kernel's own PMC entry
    traffic = load_traffic(a.config, mode, world, variant, K_loc)
    parallelism = {"single": "1 GPU",
                   "client": f"client-axis x{world}: {K_total} clients, ~{K_total // world} per GPU, fp32 partial + "
                             f"RCCL reduce-scatter, {a.chunks}-chunk pipeline",
                   "param": f"parameter-axis x{world}: every GPU holds its whole keys of all {K_total} clients "
                            f"(fedml_amd.multidev.shard_plan), no collective, bit-exact"}[mode]
    if weak:
        parallelism += f" [weak: {K} clients per GPU]"
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "client-params/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "int64" if a.op in ("secagg", "lsa") else "bf16" if dom_dt == torch.bfloat16 else "f32",
        "data": "synthetic (base~N(0,0.05^2), client=base+0.01*eps, generated in HBM)",
        "config": {
            "workload": cfg["desc"] + (f" [--clients {K}]" if a.clients is not None else ""),
            "clients_per_gpu": K_loc,
            "clients_total": K_total,
            "elements_per_client": n_elems,
            "layout": "ClientBucket rows [K, L] per dtype, 256-B aligned rows",
            "low_precision_acc": a.acc,
            "server_step": ({"sgd": "SGD lr=1.0 momentum=0.9", "adam": "Adam lr=1.0 betas=(0.9,0.999)",
                             "adagrad": "Adagrad lr=1.0 eps=1e-10",
                             "adamw": "AdamW lr=1.0 weight_decay=0.01",
                             "rmsprop": "RMSprop lr=1.0 alpha=0.99"}[a.fedopt]
                            + (" fused" if server is not None else
                               f", on each rank's 1/{world} shard after the reduce-scatter, sharded state")
                            if a.fedopt else None),
            "parallelism": parallelism,
        },
        "roofline": {
            "bound": "valu" if a.op == "krum" and not gram_op else "hbm",
            "achieved": round(achieved / 1e3, 2) if a.op == "krum" and not gram_op else round(achieved, 1),
            "peak": VALU_PEAK_TFLOPS if a.op == "krum" and not gram_op else HBM_PEAK_GBPS,
            "unit": "TFLOP/s" if a.op == "krum" and not gram_op else "GB/s",
            "frac": round(achieved / 1e3 / VALU_PEAK_TFLOPS if a.op == "krum" and not gram_op
                          else achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "kernel": ({"secagg": "reduce_kernel<OpSumModI64>", "lsa": "reduce_kernel<OpWrapSumI64, LsaEpi>",
                        "krum": ((f"pairgram_split8_kernel<{(K + 15) // 16}> + gram_sum_kernel + gram_dist_kernel "
                                  "(centred Gram, exact 3-way bf16 split, 16x16x32 bf16 MFMA)") if a.pair_distance == "gram" or
                                 (a.pair_distance == "auto" and K <= 128) else
                                 ("pairtri_kernel<16> + tri_finish_kernel" if K <= 64 else
                                  "pairtri_kernel<32> + tri_finish_kernel" if K <= 128 else
                                  "pairdist_kernel + pair_finish_kernel") + " (packed fp32)"),
                        "dist2": "dist2_kernel + sum_rows_kernel",
                        "clip": "clip_diff_kernel", "rlr": "reduce_kernel<OpF32Rlr, RlrEpi>",
                        "mpi": "reduce_kernel<OpF32MulDiv> (fl(fl(p n_i) / N))"}[a.op]
                       if a.op in ("secagg", "lsa", "krum", "dist2", "clip", "rlr", "mpi") else
                       median_kernel_name(K, dom_dt) if a.op == "median" else
                       ({"adam": "reduce_fused_kernel<OpF32,AdamEpi>", "adamw": "reduce_fused_kernel<OpF32,AdamEpi>",
                         "adagrad": "reduce_kernel<OpF32,AdagradEpi>", "rmsprop": "reduce_kernel<OpF32,AdagradEpi>"}
                        .get(a.fedopt, "reduce_kernel<OpF32,SgdEpi>"))
                       + " (FedAvg+server step fused)"
                       if server is not None else
                       f"reduce_kernel<OpF32> x{n_launch}/step + shard step" if sharded_opt is not None else
                       f"reduce_kernel<{'OpF32' if dom_dt == torch.float32 else dom_dt}> x{n_launch}/step"),
            "alg_bytes_per_step": dom_bytes,
            "kernel_ms_per_step": round(kern_ms, 4),
            **({"useful_tflops": round(krum_pair_flops / (kern_ms / 1e3) / 1e12, 2),
                # NT 16x16 tiles x 12 MFMAs of 16 cycles per 64 columns, over 1024 SIMDs at 2.4 GHz
                "bf16_mfma_floor_ms": round(((K + 15) // 16) * ((K + 15) // 16 + 1) // 2 * 12 * 16 * (n_weight / 64)
                                            / (1024 * 2.4e9) * 1e3, 3)}
               if gram_op else {}),
        },
        "cpu_baseline": None,
    }
    if a.op == "median":
        # the sorting networks are VALU-bound above ~128 clients: their min / max /
        # med3 / DPP ops issue at 4 cycles per wave64 instruction per SIMD
        # (tools/valu_rate_probe.hip), so this is the share of the SIMDs' issue
        # capacity the kernel's executed VALU instructions take
        vv = load_median_valu(a.config, mode, world, variant, K_loc)
        if vv:
            issue_ms = vv["valu_instr_per_wave"] * vv["waves_per_launch"] * VALU_HALF_RATE_CYCLES / (
                SIMDS * CLOCK_GHZ * 1e9) * 1e3
            line["roofline"]["valu"] = {
                "bound": "valu issue (half-rate ops, 4 cycles per wave64 instruction per SIMD)",
                "instr_per_wave": vv["valu_instr_per_wave"], "waves_per_launch": vv["waves_per_launch"],
                "issue_ms_at_peak": round(issue_ms, 4), "frac": round(issue_ms / kern_ms, 4),
                "source": "profiles/median_valu.json (SQ_INSTS_VALU / SQ_WAVES)"}
    if world > 1:
        # whole-job HBM rate: every rank's algorithmic bytes over the step time
        line["roofline"]["aggregate_gbps"] = round(hbm_all, 1)
        line["roofline"]["aggregate_frac_of_n_peaks"] = round(hbm_all / (world * HBM_PEAK_GBPS), 4)
        if mode == "client":
            line["exchange"] = {"mode": "client", "backend": dist.get_backend(), "world_size": world,
                                "collective": "reduce_scatter_tensor (RCCL)" if a.backend == "nccl" else "gloo (host)",
                                "xgmi_bytes_per_rank_per_step": xgmi_bytes,
                                "comm_ms_per_step": round(comm_ms, 4) if comm_ms is not None else None,
                                "note": "comm_ms: mean over ranks of the chunks' reduce-scatter time on the comm "
                                        "stream (overlapping the next chunk's reduction)"}
        elif mode == "param" and a.op == "fedavg" and not a.fedopt:
            # the headline is the exchange-free parameter axis of N processes;
            # two more measurements on the same clients follow, each after this
            # rank's rows are freed
            del step, outs, gd, groups, bucket
            torch.cuda.empty_cache()
            if not a.no_exchange:
                # north_star's client axis + RCCL reduce-scatter over xGMI
                try:
                    line["exchange"] = measure_client_axis(a, entries, n_elems, K_total, world, rank, dev)
                except Exception as e:  # the headline above stands; report what the nested run hit
                    line["exchange"] = {"mode": "client", "error": f"{type(e).__name__}: {e}"}
            if not a.no_inprocess:
                # FedML's server is ONE process: rank 0 alone drives all N
                # GPUs through the multi-device bucket while the others wait
                torch.cuda.synchronize()
                host_barrier("inprocess_start", world)
                if rank == 0:
                    try:
                        line["inprocess"] = measure_inprocess(a, entries, n_elems, K_total, world)
                    except Exception as e:
                        line["inprocess"] = {"error": f"{type(e).__name__}: {e}"}
                host_barrier("inprocess_end", world)
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.op == "fedavg":  # the reference's FedAvg loop
        line["cpu_baseline"] = cpu_baseline(bucket, ns_local, a.cpu_reps)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
