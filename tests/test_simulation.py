"""fedml_amd.simulation.fedavg_aggregate: the SP simulators' _aggregate
(sp/fedavg/fedavg_api.py:144-159) — host-side contract without a GPU, and
the reduction itself on the GPU against the oracle."""
from __future__ import annotations

import copy
from collections import OrderedDict

import pytest
import torch

import golden_util as gu
from fedml_amd import shapes
from fedml_amd.simulation import fedavg_aggregate
from fedml_amd.synth import host_clients
from oracle import fedavg_oracle as orc


def test_contract_errors_without_gpu():
    d = OrderedDict(w=torch.ones(2))
    with pytest.raises(ZeroDivisionError):
        fedavg_aggregate([(0, d), (0, OrderedDict(w=torch.ones(2)))])
    with pytest.raises(ValueError):
        fedavg_aggregate([(1, d, None)])
    with pytest.raises(IndexError):
        fedavg_aggregate([])
    empty = OrderedDict()
    assert fedavg_aggregate([(0, empty)]) is empty  # no keys: nothing divides by zero


class _A:
    federated_optimizer = "FedAvg"


@pytest.mark.gpu
@pytest.mark.parametrize("on_device", [False, True])
def test_matches_reference_fedavg(on_device, cuda_device):
    raw = host_clients(shapes.MODELS["cnn_web"](), 5, seed=8, round_idx=1)
    exp = orc.agg(_A(), copy.deepcopy(raw))
    if on_device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    first = raw[0][1]
    res = fedavg_aggregate(raw)
    assert res is first
    for k in exp:
        assert res[k].is_cuda == on_device
        gu.assert_same(res[k].cpu(), exp[k], k)


MPI = [c["name"] for c in __import__("cases").MPI_CASES]


def _to_device_aliased(raw, dev):
    memo = {}

    def move(d):
        if id(d) not in memo:
            memo[id(d)] = OrderedDict((k, t.to(dev)) for k, t in d.items())
        return memo[id(d)]

    return [(item[0],) + tuple(move(d) for d in item[1:]) for item in raw]


@pytest.mark.gpu
@pytest.mark.parametrize("name", MPI)
@pytest.mark.parametrize("where", ["host", "device"])
def test_mpi_order_matches_reference(name, where, cuda_device):
    """fedavg_mpi_aggregate = FedAVGAggregator._fedavg_aggregation_
    (simulation/mpi/fedavg/FedAVGAggregator.py:99-116) bit for bit, on host
    and device dicts, through fedagg_wsum_muldiv."""
    import cases
    from fedml_amd.simulation import fedavg_mpi_aggregate

    meta, arrays = gu.load(name)
    raw = cases.build_inputs(meta["spec"])
    if where == "device":
        raw = _to_device_aliased(raw, cuda_device)
    first = raw[0][1]
    res = fedavg_mpi_aggregate(raw)
    assert res is first
    for t in res.values():
        assert t.device.type == ("cuda" if where == "device" else "cpu")
    gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


def test_mpi_contract_without_gpu():
    from fedml_amd.simulation import fedavg_mpi_aggregate

    with pytest.raises(ValueError):
        fedavg_mpi_aggregate([(1, OrderedDict(w=torch.ones(2)), None)])
    empty = OrderedDict()
    assert fedavg_mpi_aggregate([(0, empty)]) is empty


def test_mpi_weight_records():
    """The weight records fedagg_wsum_muldiv reads (include/fedagg.h): fl32 of
    the Python scalars as torch converts them, int64 n with its flag."""
    import numpy as np

    from fedml_amd import kernels as kn

    assert kn.scalar_f32(2 ** 24 + 1) == 2 ** 24  # int64 -> float: RNE
    assert kn.scalar_f32(0.1) == float(np.float32(0.1))
    rec = kn._MULDIV_I
    assert rec.itemsize == 24 and kn._MULDIV_F.itemsize == 8 and kn._MULDIV_D.itemsize == 16
    assert [rec.fields[f][1] for f in ("n", "nf", "d", "is_int")] == [0, 8, 12, 16]


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", [(3, 1), (5, 4099), (17, 70_001), (64, 1_048_577), (9, 4_194_304)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64])
def test_muldiv_kernel_every_tile_vs_oracle(K, N, dtype, cuda_device):
    """fedagg_wsum_muldiv on device tensors across the tile configs (small,
    mid, shipped tiles and their ragged edges), aligned and at a one-element
    offset, integer and float sample counts, against the oracle's
    element-wise restatement of `p * n / N` (oracle.mpi_fedavg)."""
    from fedml_amd.simulation import fedavg_mpi_aggregate

    g = torch.Generator(device=cuda_device).manual_seed(K * 7919 + N)

    def make(n):
        if dtype == torch.int64:
            return torch.randint(-(2 ** 40), 2 ** 40, (n,), generator=g, device=cuda_device)
        return (torch.randn(n, generator=g, device=cuda_device) * 0.05).to(dtype)

    for offset in (0, 1):
        ns = [(10 ** 7 + 13 * i) if i % 2 else (3.5 + i) for i in range(K)]  # ints (int64 products wrap) and floats
        raw = [(ns[i], OrderedDict(x=make(N + offset)[offset:])) for i in range(K)]
        host = [(n, OrderedDict(x=d["x"].cpu())) for n, d in raw]
        exp = orc.mpi_fedavg(host)["x"]
        got = fedavg_mpi_aggregate(raw)["x"]
        gu.assert_same(got.cpu(), exp, f"K={K} N={N} {dtype} offset={offset}")


SP_ALIAS = [c["name"] for c in __import__("cases").ALIAS_CASES if c["optimizer"] in ("FedAvg", "FedProx")
            and not c.get("tensor_alias")]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SP_ALIAS)
@pytest.mark.parametrize("where", ["host", "device"])
def test_sp_aggregate_alias_matches_reference(name, where, cuda_device):
    """FedAvgAPI._aggregate (fedavg_api.py:144-159) is the same rebind-then-+=
    loop as the plugin's FedAvg / FedProx branch, so client 0's dict listed
    again reads the running sum there too: the FedAvg / FedProx alias
    fixtures, produced by the reference's own loop, bit for bit through
    fedavg_aggregate on host and device dicts."""
    import cases

    meta, arrays = gu.load(name)
    raw = cases.build_inputs(meta["spec"])
    if where == "device":
        raw = _to_device_aliased(raw, cuda_device)
    first = raw[0][1]
    res = fedavg_aggregate(raw)
    assert res is first
    gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


def test_sp_aggregate_alias_known_answer_contract():
    """Host-side: the alias program is taken (no GPU needed to decide it) --
    [(1, d), (1, d), (2, e)] reads the running sum at index 1."""
    from fedml_amd.agg_operator import _reads_running_cell

    d, e = OrderedDict(w=torch.tensor([1.0, 2.0])), OrderedDict(w=torch.tensor([3.0, 4.0]))
    assert _reads_running_cell([(1, d), (1, d), (2, e)], (1,))
    assert not _reads_running_cell([(1, d), (1, OrderedDict(d)), (2, e)], (1,))
