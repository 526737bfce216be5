"""Two ranks sharing the one GPU of the box (gloo, host-staged collectives):
the client-axis and parameter-axis modes with the real HIP kernels.

RCCL refuses two ranks on one device, so this rehearses everything of the
multi-GPU path except RCCL itself (the driver's 8-GPU run covers that).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import traceback

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(K, L):
    g = torch.Generator().manual_seed(11)
    return torch.randn(K, L, generator=g) * 0.05


def _worker(rank, world, port, K_local, L, q):
    try:
        import torch.distributed as dist

        from fedml_amd.sharded import ClientAxisAggregator, ParamAxisAggregator, shard_range

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda:0")
        K = K_local * world
        allrows = _rows(K, L)
        ns = list(range(100, 100 + K))
        ws = [n / sum(ns) for n in ns]
        rows = torch.zeros(K_local, (L + 63) // 64 * 64, device=dev)
        rows[:, :L] = allrows[rank * K_local:(rank + 1) * K_local].to(dev)
        agg = ClientAxisAggregator(rows, L, chunks=3)
        agg.aggregate(ws[rank * K_local:(rank + 1) * K_local])
        full = agg.gather_full().cpu()
        lo, hi = shard_range(L, world, rank)
        prows = torch.zeros(K, (hi - lo + 63) // 64 * 64, device=dev)
        prows[:, :hi - lo] = allrows[:, lo:hi].to(dev)
        pshard = ParamAxisAggregator(prows, hi - lo).aggregate(ws).cpu()
        q.put((rank, full.numpy(), (lo, hi, pshard.numpy()), None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put((rank, None, None, traceback.format_exc()))


def test_two_ranks_one_gpu(cuda_device):
    from oracle import fedavg_oracle as orc

    world, K_local, L = 2, 6, 200_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K_local, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, full, pshard, err = q.get(timeout=300)
        assert err is None, err
        res[r] = (full, pshard)
    for p in procs:
        p.join(timeout=60)
    K = K_local * world
    allrows = _rows(K, L)
    ns = list(range(100, 100 + K))
    ws = [n / sum(ns) for n in ns]
    chain = orc.wsum([allrows[i] for i in range(K)], ws).numpy()
    p0 = orc.wsum([allrows[i] for i in range(K_local)], ws[:K_local]).numpy()
    p1 = orc.wsum([allrows[i] for i in range(K_local, K)], ws[K_local:]).numpy()
    for r in range(world):
        full, (lo, hi, ps) = res[r]
        assert np.array_equal(full.view(np.uint32), (p0 + p1).view(np.uint32))  # one rounding per element
        assert np.array_equal(ps.view(np.uint32), chain[lo:hi].view(np.uint32))  # param axis: bit-exact


def _rccl_worker(port, L, q):
    """One rank, RCCL backend: ClientAxisAggregator with the process group
    handed in takes the collective path (comm stream, async
    reduce_scatter_tensor, work.wait(), stream join) and all_gather."""
    try:
        import torch.distributed as dist

        from fedml_amd.sharded import ClientAxisAggregator, ShardedFedOpt
        from oracle import fedavg_oracle as orc

        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        group = dist.group.WORLD
        calls = {"rs": 0, "ag": 0}
        rs, ag = dist.reduce_scatter_tensor, dist.all_gather

        def count_rs(*a, **k):
            calls["rs"] += 1
            return rs(*a, **k)

        def count_ag(*a, **k):
            calls["ag"] += 1
            return ag(*a, **k)

        dist.reduce_scatter_tensor, dist.all_gather = count_rs, count_ag
        K = 7
        host = _rows(K, L)
        ws = [(i + 1.0) / 28.0 for i in range(K)]
        chain = orc.wsum([host[i] for i in range(K)], ws).numpy()
        rows = torch.zeros(K, (L + 63) // 64 * 64, device=dev)
        rows[:, :L] = host.to(dev)
        out = {}
        for chunks in (1, 3, 8):
            agg = ClientAxisAggregator(rows, L, group=group, chunks=chunks)
            assert agg.collective and agg.comm_stream is not None and not agg.host_staged
            before = calls["rs"]
            agg.aggregate(ws)
            out[chunks] = agg.gather_full().cpu().numpy()
            assert calls["rs"] - before == len(agg.bounds)
        # the sharded FedOpt on the same group (step after the exchange)
        sh = ShardedFedOpt(rows, L, torch.zeros(L, device=dev), "sgd", 1.0, 0.9, group=group, chunks=3)
        sh.aggregate(ws)
        p1 = sh.gather_params().cpu().numpy()
        torch.cuda.synchronize()
        backend = dist.get_backend()
        dist.destroy_process_group()
        q.put((out, chain, p1, calls, backend, None))
    except Exception:  # pragma: no cover
        q.put((None, None, None, None, None, traceback.format_exc()))


def test_rccl_branch_one_rank(cuda_device):
    """The RCCL (NCCL backend) path of the client-axis mode, executed: a
    one-rank process group on the box's GPU.  Results are bit-exact with the
    single chain for 1, 3 and 8 chunks (one rank: the reduce-scatter is the
    identity), and the first SGD step (lr 1, fresh momentum) returns the
    average itself."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    L = 300_007
    p = ctx.Process(target=_rccl_worker, args=(_port(), L, q))
    p.start()
    out, chain, p1, calls, backend, err = q.get(timeout=300)
    p.join(timeout=60)
    assert err is None, err
    assert backend == "nccl"
    assert calls["rs"] >= 1 + 3 + 8 and calls["ag"] >= 4
    for chunks, full in out.items():
        assert np.array_equal(full.view(np.uint32), chain.view(np.uint32)), chunks
    # SGD lr=1, first step: p_new = fl(p_old - fl(p_old - avg)) with p_old = 0 -> avg
    assert np.array_equal(p1.view(np.uint32), chain.view(np.uint32))


def _bf16_worker(rank, world, port, K_local, L, q):
    """Config 4's split with the real kernels: this rank's bf16 rows ->
    fedagg_wsum_bf16_f32out (fp32 partial, GLOBAL weights) -> gloo
    reduce-scatter -> shard_in_model_dtype (one bf16 rounding) -> gather."""
    try:
        import torch.distributed as dist

        from fedml_amd.sharded import ClientAxisAggregator

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda:0")
        K = K_local * world
        allrows = _rows(K, L).to(torch.bfloat16)
        ns = list(range(100, 100 + K))
        ws = [n / sum(ns) for n in ns]
        rows = torch.zeros(K_local, (L + 63) // 64 * 64, device=dev, dtype=torch.bfloat16)
        rows[:, :L] = allrows[rank * K_local:(rank + 1) * K_local].to(dev)
        agg = ClientAxisAggregator(rows, L, chunks=3)
        agg.aggregate(ws[rank * K_local:(rank + 1) * K_local])
        part32 = agg.gather_full().cpu()
        full16 = agg.gather_full(agg.shard_in_model_dtype()).cpu()
        q.put((rank, part32.numpy(), full16.view(torch.int16).numpy(), None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world,K_local", [(2, 64), (4, 32)])
def test_two_and_four_ranks_bf16_split(world, K_local, cuda_device):
    """The bf16 client-axis path at world 2 and 4 with the HIP kernel (no
    numpy stand-in): each rank's fp32 partial is exactly the fp32 chain of its
    clients' fl(w_i p_i); the exchange sums them; the result is that sum
    rounded ONCE to bf16.  For two ranks that is bit-exact against
    bf16(fl(p0 + p1)); at any world it is within DESIGN §2's bound of the
    reference's own bf16 chain (a bf16 rounding after every mul and add)."""
    from oracle import fedavg_oracle as orc

    L = 100_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bf16_worker, args=(r, world, port, K_local, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, part32, full16, err = q.get(timeout=300)
        assert err is None, err
        res[r] = (part32, full16)
    for p in procs:
        p.join(timeout=60)
    K = K_local * world
    rows16 = _rows(K, L).to(torch.bfloat16)
    rows32 = rows16.to(torch.float32)
    ns = list(range(100, 100 + K))
    ws = [n / sum(ns) for n in ns]
    parts = [orc.wsum([rows32[i] for i in range(r * K_local, (r + 1) * K_local)], ws[r * K_local:(r + 1) * K_local])
             for r in range(world)]
    for r in range(world):
        part32, full16 = res[r]
        assert np.array_equal(res[0][1], full16)  # every rank gathers the same model
        if world == 2:
            want32 = (parts[0] + parts[1]).numpy()
            assert np.array_equal(part32.view(np.uint32), want32.view(np.uint32))
            want16 = torch.from_numpy(want32).to(torch.bfloat16).view(torch.int16).numpy()
            assert np.array_equal(full16, want16)
    got = torch.from_numpy(res[0][1]).view(torch.bfloat16).to(torch.float64)
    # against the exact sum: T (fp32 reorder) + half a bf16 ulp + the products' fp32 roundings
    prods = torch.stack([(rows32[i] * ws[i]).to(torch.float64) for i in range(K)])
    exact = (rows32.to(torch.float64) * torch.tensor(ws, dtype=torch.float64)[:, None]).sum(0)
    s_abs = prods.abs().sum(0)
    from fedml_amd.sharded import ClientAxisAggregator

    T = ClientAxisAggregator.tolerance(s_abs, K, world)
    assert torch.all((got - exact).abs() <= T + 2.0 ** -8 * exact.abs() + 2.0 ** -24 * K * s_abs)
    # against the reference's bf16 chain (agg_operator.py:40-44): within its own error bound of exact as well
    ref = orc.wsum([rows16[i] for i in range(K)], ws).to(torch.float64)
    run = torch.zeros(L, dtype=torch.float64)
    bound = torch.zeros(L, dtype=torch.float64)
    for i in range(K):
        run = run + prods[i]
        bound += run.abs()
    bound = 2.0 ** -8 * (bound + s_abs)
    assert torch.all((got - ref).abs() <= bound + T + 2.0 ** -8 * exact.abs() + 2.0 ** -24 * K * s_abs)
