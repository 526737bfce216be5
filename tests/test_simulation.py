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
