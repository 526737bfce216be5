"""Client-axis aggregation over RCCL with 2 ranks (tool; launched by torchrun).

On a 1-GPU box both ranks share cuda:0 (RCCL may refuse that: then this probe
just reports the refusal).  Checks the reduce-scatter result against the
single-chain oracle within ClientAxisAggregator.tolerance.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from fedml_amd.sharded import ClientAxisAggregator  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    K_local, L = 8, 1_000_003
    g = torch.Generator().manual_seed(5)
    allrows = torch.randn(K_local * world, L, generator=g) * 0.05
    ns = [int(v) for v in np.random.default_rng(3).integers(100, 1001, K_local * world)]
    ws = [n / sum(ns) for n in ns]
    rows = torch.zeros(K_local, (L + 63) // 64 * 64, device=dev)
    rows[:, :L] = allrows[rank * K_local:(rank + 1) * K_local].to(dev)
    agg = ClientAxisAggregator(rows, L, chunks=4)
    agg.aggregate(ws[rank * K_local:(rank + 1) * K_local])
    full = agg.gather_full().cpu().double()
    chain = torch.zeros(L, dtype=torch.float32)
    for i in range(K_local * world):
        t = allrows[i] * ws[i]
        chain = t if i == 0 else chain + t
    terms = sum((allrows[i].double() * np.float32(ws[i])).abs() for i in range(K_local * world))
    bound = ClientAxisAggregator.tolerance(terms, K_local * world, world)
    err = (full - chain.double()).abs()
    ok = bool((err <= bound).all())
    print(f"rank {rank}: world {world} on {ndev} device(s): max err {float(err.max()):.3e} "
          f"bound ok={ok}", flush=True)
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
