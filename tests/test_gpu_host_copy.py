"""fedml_amd.host_copy.to_host: the averaged model back to the host one DMA
per result buffer, bit-identical to per-key .cpu(); and the server
aggregator's set_model_params into a host model, identical to
load_state_dict (default_aggregator.py:25-27)."""
from __future__ import annotations

from collections import OrderedDict

import pytest
import torch

from fedml_amd.agg_operator import FedMLAggOperator
from fedml_amd.host_copy import to_host
from fedml_amd.server_aggregator import MI355XServerAggregator


def _bits_equal(a: torch.Tensor, b: torch.Tensor) -> bool:
    return a.dtype == b.dtype and a.shape == b.shape and torch.equal(a.reshape(-1).view(torch.uint8),
                                                                       b.reshape(-1).view(torch.uint8))


def test_host_values_pass_through():
    t = torch.arange(6.0)
    out = to_host(OrderedDict(a=t, n=3, b=torch.zeros(0)))
    assert out["a"] is t and out["n"] == 3 and out["b"].numel() == 0


class _A:
    federated_optimizer = "FedAvg"


def _round(dev, K=5):
    g = torch.Generator(device=dev).manual_seed(3)
    keys = [("w", (64, 33), torch.float32), ("b", (33,), torch.float32), ("n", (), torch.int64),
            ("h", (17, 4), torch.bfloat16), ("e", (0,), torch.float32), ("c", (7,), torch.int64)]
    raw = []
    for i in range(K):
        d = OrderedDict()
        for k, s, dt in keys:
            if dt == torch.int64:
                d[k] = torch.randint(0, 100, s, generator=g, device=dev)
            else:
                d[k] = torch.randn(s, generator=g, device=dev).to(dt)
        raw.append((i + 1, d))
    return raw


@pytest.mark.gpu
def test_to_host_of_an_aggregated_round_is_per_key_cpu(cuda_device):
    avg = FedMLAggOperator.agg(_A(), _round(cuda_device))
    avg["extra"] = torch.randn(9, device=cuda_device)  # its own allocation
    avg["strided"] = torch.randn(8, 6, device=cuda_device)[:, ::2]  # not contiguous
    avg["host"] = torch.ones(3)
    avg["meta"] = "x"
    ref = OrderedDict((k, v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in avg.items())
    out = to_host(avg)
    assert list(out) == list(avg)
    for k, v in ref.items():
        if isinstance(v, torch.Tensor):
            assert not out[k].is_cuda and _bits_equal(out[k], v), k
        else:
            assert out[k] == v


@pytest.mark.gpu
def test_to_host_writes_into_matching_host_tensors(cuda_device):
    avg = FedMLAggOperator.agg(_A(), _round(cuda_device))
    into = OrderedDict((k, torch.empty(v.shape, dtype=v.dtype)) for k, v in avg.items())
    into["n"] = torch.zeros((), dtype=torch.int64)  # the model's counter: int64, the average float32
    keep = {k: v for k, v in into.items()}
    out = to_host(avg, into=into)
    for k, v in avg.items():
        assert _bits_equal(out[k], v.cpu()), k
        if v.numel():  # (an empty key is returned as a fresh empty tensor)
            assert (out[k] is keep[k]) == (keep[k].dtype == v.dtype), k


@pytest.mark.gpu
def test_sparse_views_of_a_big_buffer_go_key_by_key(cuda_device):
    big = torch.randn(1 << 20, device=cuda_device)
    sd = OrderedDict(a=big[:5], b=big[-7:])  # 48 bytes used of a 4 MB span
    out = to_host(sd)
    assert _bits_equal(out["a"], big[:5].cpu()) and _bits_equal(out["b"], big[-7:].cpu())


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(33, 64)
        self.bn = torch.nn.BatchNorm1d(64)


@pytest.mark.gpu
def test_set_model_params_into_a_host_model_is_load_state_dict(cuda_device):
    net = _Net()
    K = 4
    g = torch.Generator(device=cuda_device).manual_seed(5)
    raw = []
    for i in range(K):
        d = OrderedDict()
        for k, v in net.state_dict().items():
            if v.dtype == torch.int64:
                d[k] = torch.randint(0, 50, v.shape, generator=g, device=cuda_device)
            else:
                d[k] = torch.randn(v.shape, generator=g, device=cuda_device)
        raw.append((10 + i, d))
    avg = FedMLAggOperator.agg(_A(), raw)
    assert avg["bn.num_batches_tracked"].dtype == torch.float32  # int64 * float -> float32, as the reference
    ref = _Net()
    ref.load_state_dict(avg)
    agg = MI355XServerAggregator(net, _A())
    before = {k: v.data_ptr() for k, v in net.state_dict().items()}
    agg.set_model_params(avg)
    for k, v in ref.state_dict().items():
        got = net.state_dict()[k]
        assert _bits_equal(got, v), k
        assert got.data_ptr() == before[k], k  # written in place, as load_state_dict does


class _Scaled(torch.nn.Linear):
    """A module that transforms values on load (its own _load_from_state_dict)."""

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        state_dict = {k: (v * 2 if k.startswith(prefix) else v) for k, v in state_dict.items()}
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


def test_plain_load_detects_load_overrides_and_hooks():
    """CPU: the in-place fast path is taken only when load_state_dict would
    only copy: torch's BatchNorm override is benign, a custom
    override or a load hook is not."""
    from fedml_amd.server_aggregator import _plain_load

    assert _plain_load(_Net())
    assert not _plain_load(torch.nn.Sequential(torch.nn.Linear(2, 2), _Scaled(2, 2)))
    m = torch.nn.Sequential(torch.nn.Linear(2, 2))
    m[0].register_load_state_dict_post_hook(lambda module, keys: None)
    assert not _plain_load(m)


@pytest.mark.gpu
def test_set_model_params_runs_load_overrides_and_bumps_versions(cuda_device):
    """A model whose module transforms values on load gets what
    load_state_dict gives it; the in-place fast path bumps the parameters'
    version counters as load_state_dict's copy_ does."""
    net = torch.nn.Sequential(torch.nn.Linear(8, 4), _Scaled(4, 2))
    raw = [(1 + i, OrderedDict((k, torch.randn(v.shape, device=cuda_device)) for k, v in net.state_dict().items()))
           for i in range(3)]
    avg = FedMLAggOperator.agg(_A(), raw)
    ref = torch.nn.Sequential(torch.nn.Linear(8, 4), _Scaled(4, 2))
    ref.load_state_dict(OrderedDict((k, v.cpu()) for k, v in avg.items()))
    MI355XServerAggregator(net, _A()).set_model_params(avg)
    for k, v in ref.state_dict().items():
        assert _bits_equal(net.state_dict()[k], v), k
    plain = _Net()
    raw = [(1 + i, OrderedDict((k, (torch.randn(v.shape) if v.is_floating_point() else v.clone()).to(cuda_device))
                               for k, v in plain.state_dict().items())) for i in range(2)]
    avg = FedMLAggOperator.agg(_A(), raw)
    versions = {k: v._version for k, v in plain.state_dict().items()}
    MI355XServerAggregator(plain, _A()).set_model_params(avg)
    for k, v in plain.state_dict().items():
        assert v._version > versions[k], k
