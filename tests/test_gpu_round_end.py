"""GPU: the pipelined round end (ClientBucket.reduce_to_host) — chunked
reduction, D2H on a copy stream and the host scatter overlapped — against
reduce_into + to_host and the oracle, bit for bit."""
from __future__ import annotations

from collections import OrderedDict

import pytest
import torch

import golden_util as gu
from fedml_amd.bucket import ClientBucket
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


def _layout(n_big: int):
    """fp32 weights of ragged sizes (several straddle the chunk bounds), int64
    counters promoted into the fp32 row, a scalar and an empty key."""
    return [("conv.weight", (n_big,), torch.float32), ("bn.num_batches_tracked", (), torch.int64),
            ("fc.weight", (1000, 77), torch.float32), ("empty", (0,), torch.float32),
            ("fc.bias", (1001,), torch.float32), ("tail", (70_001,), torch.float32),
            ("steps", (3,), torch.int64)]


def _clients(layout, K, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(K):
        d = OrderedDict()
        for k, s, dt in layout:
            if dt == torch.int64:
                d[k] = torch.randint(0, 1 << 40, s, generator=g, dtype=torch.int64)
            else:
                d[k] = torch.randn(s, generator=g) * 0.05
        out.append((float(10 + 3 * i), d))
    return out


def _expected(raw):
    ns = [n for n, _ in raw]
    w = [n / sum(ns) for n in ns]
    return {k: orc.wsum([d[k] for _, d in raw], w) for k in raw[0][1]}, w


@pytest.mark.parametrize("chunks", [1, 3, 8])
@pytest.mark.parametrize("n_big", [5, 300_000, 2_000_003])
def test_reduce_to_host_matches_oracle(chunks, n_big, cuda_device):
    layout = _layout(n_big)
    K = 9
    raw = _clients(layout, K, seed=n_big + chunks)
    exp, w = _expected(raw)
    bucket = ClientBucket(layout, K, cuda_device)
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    first = bucket.reduce_to_host(w, chunks=chunks)
    assert list(first) == [k for k, _, _ in layout]
    for k, t in first.items():
        assert not t.is_cuda and t.dtype == torch.float32 and tuple(t.shape) == tuple(exp[k].shape), k
        gu.assert_same(t, exp[k], f"chunks={chunks} {k}")
    # the serial path gives the same bits
    outs = bucket.new_outputs()
    bucket.reduce_into(outs, w)
    serial = bucket.to_host(outs)
    for k in first:
        gu.assert_same(first[k], serial[k], f"serial {k}")
    # a second call (pooled, pre-touched tensors) returns NEW tensors and
    # leaves the first call's results alone
    keep = {k: t.clone() for k, t in first.items()}
    second = bucket.reduce_to_host(w, chunks=chunks)
    for k in first:
        assert second[k].data_ptr() != first[k].data_ptr() or first[k].numel() == 0, k
        gu.assert_same(second[k], exp[k], f"second {k}")
        gu.assert_same(first[k], keep[k], f"first kept {k}")


def test_reduce_to_host_into_and_fewer_clients(cuda_device):
    layout = _layout(1_000_000)
    K = 6
    raw = _clients(layout, K, seed=11)
    bucket = ClientBucket(layout, K + 3, cuda_device)  # capacity above the round's client count
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    exp, w = _expected(raw)
    into = OrderedDict((k, torch.full(s, -1.0)) for k, s, _ in layout)
    res = bucket.reduce_to_host(w, num_clients=K, into=into, chunks=4)
    for k in exp:
        assert res[k] is into[k], k
        gu.assert_same(res[k], exp[k], k)
    with pytest.raises(ValueError):
        bucket.reduce_to_host(w[:-1], num_clients=K)


def test_reduce_to_host_bf16_model_with_fp32_keys(cuda_device):
    """A bf16 model whose norms stay fp32: the bf16 group is chunked, the fp32
    group follows; both bit-exact in the reference chain."""
    layout = [("w", (1_500_007,), torch.bfloat16), ("norm", (4099,), torch.float32),
              ("w2", (70_001,), torch.bfloat16)]
    K = 17
    g = torch.Generator().manual_seed(3)
    raw = [(float(i + 1), OrderedDict((k, (torch.randn(s, generator=g) * 0.1).to(dt)) for k, s, dt in layout))
           for i in range(K)]
    exp, w = _expected(raw)
    bucket = ClientBucket(layout, K, cuda_device)
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    res = bucket.reduce_to_host(w, chunks=5)
    for k in exp:
        assert res[k].dtype == exp[k].dtype, k
        gu.assert_same(res[k], exp[k], k)


@pytest.mark.parametrize("chunks", [3, 8])
def test_reduce_to_host_waits_per_piece(chunks, cuda_device):
    """Rows of ~13.4M columns: each put() lands as 4 evented H2D pieces and
    every range of the reduction waits only for the pieces it covers.  The
    last client has a device key in the middle of the row (its host runs
    skip that piece), and the round is reduced while its H2D is in flight."""
    layout = _layout(13_400_003)
    K = 4
    raw = _clients(layout, K, seed=77 + chunks)
    raw[-1][1]["fc.weight"] = raw[-1][1]["fc.weight"].to(cuda_device)  # mixed residency, last client
    exp, w = _expected([(n, OrderedDict((k, t.cpu()) for k, t in d.items())) for n, d in raw])
    bucket = ClientBucket(layout, K, cuda_device)
    for rnd in range(2):  # the second round reuses the staging and the pieces' bookkeeping
        for i, (n, d) in enumerate(raw):
            bucket.put(i, d, n)
        got = bucket.reduce_to_host(w, chunks=chunks)
        for k, t in got.items():
            gu.assert_same(t, exp[k], f"round {rnd} {k}")
        assert not bucket._pending and not bucket._piece_events


def test_reduce_to_host_after_unpieced_ingest(cuda_device):
    """A client ingested by put_encoded (one H2D without pieces) sends the
    round end back to the full wait; results unchanged."""
    from fedml_amd import wire

    layout = _layout(5_000_001)
    K = 3
    raw = _clients(layout, K, seed=5)
    exp, w = _expected(raw)
    bucket = ClientBucket(layout, K, cuda_device)
    bucket.put(0, raw[0][1], raw[0][0])
    bucket.put_encoded(1, wire.encode(raw[1][1], raw[1][0]))
    bucket.put(2, raw[2][1], raw[2][0])
    assert bucket._pending_other
    got = bucket.reduce_to_host(w)
    for k, t in got.items():
        gu.assert_same(t, exp[k], k)
