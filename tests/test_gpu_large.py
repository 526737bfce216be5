"""Single keys past the 32-bit element and byte ranges, on the GPU (maximum
sizes): the drop-in's device-dict paths over one fp32 key of 2^31 + 12,345
elements (8.6 GB per client) and one bf16 key of 2^32 + 777 elements, checked
against the oracle on sampled columns (every element's chain is independent of
N, so the oracle runs on the gathered columns).

Paths: FedMLAggOperator.agg FedAvg (agg_operator.py:35-54), FedAvg_seq in
place (:55-63), and the MPI simulation order (FedAVGAggregator.py:99-116).
The sample holds 100,000 random columns plus the columns around 2^31, 2^32
(bf16) and the first and last 64.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import golden_util as gu
from fedml_amd.agg_operator import FedMLAggOperator
from fedml_amd.simulation import fedavg_mpi_aggregate
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


class _Args:
    def __init__(self, opt, K):
        self.federated_optimizer = opt
        self.client_num_per_round = K
        self.client_num_in_total = K


def _columns(N: int, seed: int) -> torch.Tensor:
    rng = np.random.default_rng(seed)
    picks = [rng.integers(0, N, 100_000), np.arange(64), np.arange(N - 64, N)]
    for edge in (2 ** 31, 2 ** 32):
        if edge < N:
            picks.append(np.arange(edge - 64, edge + 64))
    return torch.from_numpy(np.unique(np.concatenate(picks)))


def _clients(K: int, N: int, dtype, dev, seed: int):
    g = torch.Generator(device=dev).manual_seed(seed)
    base = torch.empty(N, dtype=dtype, device=dev).normal_(0.0, 0.05, generator=g)
    out = []
    for i in range(K):
        t = torch.empty(N, dtype=dtype, device=dev)
        t.normal_(0.0, 0.01, generator=g)
        t.add_(base)
        out.append(t)
    del base
    return out


def _gather(raw, cols):
    """The sampled columns of every client, as host dicts of the same key."""
    idx = cols.to(raw[0][1]["x"].device)
    return [(n, OrderedDict(x=d["x"][idx].cpu())) for n, d in raw]


@pytest.mark.parametrize("N,dtype", [(2 ** 31 + 12_345, torch.float32), (2 ** 32 + 777, torch.bfloat16)],
                         ids=["f32-2^31", "bf16-2^32"])
def test_key_beyond_32_bit_ranges(N, dtype, cuda_device):
    K = 3
    ns = [300, 7, 1_000_003]
    ts = _clients(K, N, dtype, cuda_device, seed=31)
    raw = [(ns[i], OrderedDict(x=ts[i])) for i in range(K)]
    cols = _columns(N, seed=5)
    small = _gather(raw, cols)
    idx = cols.to(cuda_device)

    # FedAvg through the plugin surface: one launch over the device pointers
    got = FedMLAggOperator.agg(_Args("FedAvg", K), [(n, OrderedDict(d)) for n, d in raw])["x"]
    exp = orc.agg(_Args("FedAvg", K), [(n, OrderedDict(d)) for n, d in small])["x"]
    assert got.shape == (N,) and got.dtype == dtype
    gu.assert_same(got[idx].cpu(), exp, f"FedAvg N={N} {dtype}")
    del got

    # the MPI simulation order
    got = fedavg_mpi_aggregate([(n, OrderedDict(d)) for n, d in raw])["x"]
    exp = orc.mpi_fedavg([(n, OrderedDict(d)) for n, d in small])["x"]
    gu.assert_same(got[idx].cpu(), exp, f"MPI N={N} {dtype}")
    del got

    # FedAvg_seq: adds into client 0's tensor in place
    got = FedMLAggOperator.agg(_Args("FedAvg_seq", K), raw)["x"]
    exp = orc.agg(_Args("FedAvg_seq", K), small)["x"]
    assert got.data_ptr() == ts[0].data_ptr()
    gu.assert_same(got[idx].cpu(), exp, f"FedAvg_seq N={N} {dtype}")
    del got, ts, raw
    torch.cuda.empty_cache()


@pytest.mark.parametrize("acc", ["reference", "fp32"])
@pytest.mark.parametrize("offset", [0, 1], ids=["aligned", "offset1"])
@pytest.mark.parametrize("K,N", [(256, (8 << 20) - 12_345), (300, (8 << 20) - 12_345), (40, 8 << 20),
                                 (40, (8 << 20) - 12_345)])
def test_bf16_wide_tiles(K, N, offset, acc, cuda_device):
    """bf16 over rows of 8M+ elements where the eight-packs-per-lane tiles
    run (the reference chain from 256 clients, the fp32-accumulated chain from
    32, when the last resident round is full enough: 8M - 12,345 and 8M
    elements are 512 such workgroups, two full rounds on 256 CUs), their
    ragged / unaligned edge path, and the four-pack tiles beside them.  "fp32" is fedml_amd's
    fedagg_low_precision_acc mode, checked against oracle.wsum_acc32."""
    g = torch.Generator(device=cuda_device).manual_seed(K + offset)
    L = (N + 8 + 7) // 8 * 8  # 16-byte row stride: offset 0 is aligned for every client
    rows = torch.empty((K, L), dtype=torch.bfloat16, device=cuda_device).normal_(0.0, 0.05, generator=g)
    ns = [(i % 7) + 1 for i in range(K)]
    raw = [(ns[i], OrderedDict(x=rows[i, offset:offset + N])) for i in range(K)]
    cols = _columns(N, seed=K)
    small = _gather(raw, cols)
    args = _Args("FedAvg", K)
    args.fedagg_low_precision_acc = acc
    got = FedMLAggOperator.agg(args, raw)["x"]  # device dicts: the multi-tensor launch
    ws = [n / sum(ns) for n in ns]
    if acc == "reference":
        exp = orc.agg(_Args("FedAvg", K), small)["x"]
    else:
        exp = orc.wsum_acc32([d["x"] for _, d in small], ws)
    idx = cols.to(cuda_device)
    gu.assert_same(got[idx].cpu(), exp, f"agg bf16 K={K} N={N} offset={offset} acc={acc}")
    # the single-tensor entry (fedagg_wsum_bf16: launch_ws, where the tile
    # shape is chosen by client count and last-round fill), aligned or not
    from fedml_amd import kernels as kn

    # (not from raw: agg() rebinds client 0's dict to the result, as the reference does)
    host_ptrs = [rows[i, offset:offset + N].data_ptr() for i in range(K)]
    assert kn.aligned16(host_ptrs) == (offset == 0)
    ptrs = torch.tensor(host_ptrs, dtype=torch.int64, device=cuda_device)
    out = torch.empty(N, dtype=torch.bfloat16, device=cuda_device)
    w = kn.weights_for(ws, torch.bfloat16, cuda_device)
    kn.wsum_ptrs(torch.bfloat16, ptrs, w, K, N, out, kn.aligned16(host_ptrs),
                 {"reference": kn.ACC_REFERENCE, "fp32": kn.ACC_FP32}[acc])
    gu.assert_same(out[idx].cpu(), exp, f"wsum_ptrs bf16 K={K} N={N} offset={offset} acc={acc}")
