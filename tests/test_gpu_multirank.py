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
