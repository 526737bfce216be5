"""BASELINE.json configs 4 and 5 at their own full workloads, on the GPU,
against the oracle.

config 4: FedAvg of 512 clients x ViT-B/16 (86,567,656 bf16 elements, 152
keys) — 88.6 GB of client rows, one MI355X (the 4-GPU split is the client-axis
mode of fedml_amd.sharded; here the whole round runs on one device, which is
the chain every sharding is checked against).  K is the parameter that matters
for bf16: the reference rounds to bf16 after every client.

config 5: FedAvg of 64 clients x Llama-2-7B LoRA (4,194,304 fp32) fused with
the server SGD step (lr 1.0, momentum 0.9), three rounds with the momentum
carried, every element against the C oracle (FedOptAggregator.py:93-130).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import golden_util as gu
from fedml_amd import kernels as kn
from fedml_amd import shapes
from fedml_amd.bucket import ClientBucket
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


def _fill(rows: torch.Tensor, length: int, seed: int) -> None:
    """SURVEY.md §8(d)'s synthetic clients, generated in HBM: base ~ N(0, 0.05²),
    client_i = base + 0.01·eps_i (as bench.py)."""
    g = torch.Generator(device=rows.device).manual_seed(seed)
    base = torch.randn(length, generator=g, device=rows.device) * 0.05
    eps = torch.empty(length, device=rows.device)
    for i in range(rows.shape[0]):
        eps.normal_(0.0, 1.0, generator=g)
        rows[i, :length].copy_(base + 0.01 * eps)
    del base, eps


@pytest.fixture(scope="module")
def cfg4_bucket(cuda_device):
    """512 ViT-B/16 clients in bf16 rows (88.6 GB), shared by both acc modes."""
    K = 512
    entries = shapes.vit_b16()
    assert len(entries) == 152 and shapes.numel(entries) == 86_567_656
    bucket = ClientBucket(entries, K, cuda_device)
    g = bucket.groups[torch.bfloat16]
    _fill(g.rows, g.length, seed=4)
    torch.cuda.synchronize()
    yield bucket
    del bucket, g
    torch.cuda.empty_cache()


def _sample_columns(bucket, n_random: int = 200_000) -> torch.Tensor:
    """200,000 random key elements plus the first and the last two elements
    of every key (the ragged tails of every key's tiles)."""
    g = bucket.groups[torch.bfloat16]
    rng = np.random.default_rng(12)
    ends = []
    starts = np.asarray(g.offsets, dtype=np.int64)
    counts = np.asarray(g.numels, dtype=np.int64)
    for o, n in zip(starts, counts):
        ends += [o, o + n - 2, o + n - 1]
    cum = np.cumsum(counts)
    flat = rng.choice(int(cum[-1]), n_random, replace=False)  # uniform over the model's elements
    which = np.searchsorted(cum, flat, side="right")
    rand = starts[which] + flat - (cum[which] - counts[which])
    return torch.from_numpy(np.unique(np.concatenate([rand, np.asarray(ends, dtype=np.int64)])))


@pytest.mark.parametrize("acc", ["reference", "fp32"])
def test_cfg4_vit_b16_512_clients(acc, cfg4_bucket, cuda_device):
    """Config 4 at K = 512: the bf16 FedAvg of every ViT-B/16 key through the
    bench's launch (one bf16 launch over the flat rows), bit-exact vs the
    oracle on >= 200,000 sampled columns and every key's tail.  "reference":
    torch's CPU chain (bf16 rounding after every mul and add); "fp32": fp32
    accumulation, one rounding."""
    bucket = cfg4_bucket
    bucket.acc_mode = {"reference": kn.ACC_REFERENCE, "fp32": kn.ACC_FP32}[acc]
    K = bucket.capacity
    ns = [int(v) for v in np.random.default_rng(40).integers(100, 1001, K)]
    outs = bucket.new_outputs()
    bucket.reduce_into(outs, bucket.weights(ns))
    res = bucket.unflatten(outs)
    g = bucket.groups[torch.bfloat16]
    cols = _sample_columns(bucket)
    assert cols.numel() >= 200_000
    got = outs[torch.bfloat16][cols.to(cuda_device)].cpu()
    inputs = g.rows[:, cols.to(cuda_device)].cpu()
    ws = [n / sum(ns) for n in ns]
    oracle = orc.wsum if acc == "reference" else orc.wsum_acc32
    exp = oracle([inputs[i] for i in range(K)], ws)
    gu.assert_same(got, exp, f"cfg4 K=512 {acc}")
    # the per-key views are the flat result (what the server hands back)
    last = shapes.vit_b16()[-1][0]
    assert res[last].shape == (1000,) and res[last].dtype == torch.bfloat16


def test_cfg5_fused_sgd_vs_c_oracle(cuda_device):
    """Config 5's server step at its own size: 64 clients x 4,194,304 fp32
    (LoRA r=8 q/v of Llama-2-7B), FedAvg fused with SGD lr=1.0 momentum=0.9,
    three rounds with the momentum buffer carried; parameters and momentum
    compared element for element with the C oracle (wsum chain, then the
    fmaf SGD update of FedOptAggregator.py:104-125)."""
    K = 64
    entries = shapes.llama2_7b_lora()
    N = shapes.numel(entries)
    assert N == 4_194_304
    rows = torch.empty((K, N), dtype=torch.float32, device=cuda_device)
    _fill(rows, N, seed=5)
    g = torch.Generator(device=cuda_device).manual_seed(55)
    p = torch.randn(N, generator=g, device=cuda_device) * 0.02
    mom = torch.zeros(N, device=cuda_device)
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    hp, hb = p.cpu().numpy().copy(), None
    for r in range(3):
        ns = [int(v) for v in np.random.default_rng(500 + r).integers(100, 1001, K)]
        ws = [n / sum(ns) for n in ns]
        kn.wsum_fedopt_sgd(d_ptrs, kn.weights_for(ws, torch.float32, cuda_device), K, N, p, mom, 1.0, 0.9,
                           r == 0, True)
        host = rows.cpu().numpy()
        avg = orc.c_wsum([host[i] for i in range(K)], ws)
        hp, hb = orc.fedopt_sgd(hp, avg, hb, 1.0, 0.9, r == 0)
        gu.assert_same(p.cpu(), torch.from_numpy(hp), f"round {r} param")
        gu.assert_same(mom.cpu(), torch.from_numpy(hb), f"round {r} momentum")
        rows.mul_(1.01)  # the next round's updates
