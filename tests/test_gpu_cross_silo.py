"""The cross-silo FedMLAggregator mirror (fedml_amd.cross_silo): updates
ingested into HBM on arrival, then the reference's aggregate() flow, checked
bit for bit against the oracle restatement of the reference's FedAvg."""
from __future__ import annotations

import copy
from collections import OrderedDict

import pytest
import torch

import golden_util as gu
from fedml_amd import shapes
from fedml_amd.cross_silo import FedMLAggregator
from fedml_amd.server_aggregator import MI355XServerAggregator
from fedml_amd.synth import host_clients
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


class _Args:
    federated_optimizer = "FedAvg"


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.BatchNorm1d(19), torch.nn.Linear(19, 3))


def _server(model, K, device):
    args = _Args()
    return FedMLAggregator(None, None, 0, {}, {}, {}, K, device, args, MI355XServerAggregator(model, args))


def _round(model, K, seed, round_idx):
    entries = [(k, tuple(t.shape), t.dtype) for k, t in model.state_dict().items()]
    return host_clients(entries, K, seed=seed, round_idx=round_idx)


def _keyless_server(K, device):
    """A server whose model does not carry the test's keys (set_model_params is a no-op)."""
    args = _Args()
    agg = MI355XServerAggregator(torch.nn.Linear(1, 1), args)
    agg.set_model_params = lambda p: None
    return FedMLAggregator(None, None, 0, {}, {}, {}, K, device, args, agg)


@pytest.mark.parametrize("K", [1, 3, 8])
def test_rounds_match_reference(K, cuda_device):
    """Two rounds on the same slots: each aggregate equals the reference's
    FedAvg of that round's host updates; the dicts handed over now hold device
    views with the updates' values and dtypes (what model_params_to_device
    leaves behind), and the server model holds the average."""
    model = _model().to(cuda_device)
    server = _server(model, K, cuda_device)
    for r in range(2):
        raw = _round(model, K, seed=10 + r, round_idx=r)
        exp = orc.agg(_Args(), copy.deepcopy(raw))
        for i, (n, d) in enumerate(raw):
            host_vals = OrderedDict((k, t.clone()) for k, t in d.items())
            server.add_local_trained_result(i, d, n)
            for k, t in d.items():
                assert t.is_cuda and t.dtype == host_vals[k].dtype
                gu.assert_same(t.cpu(), host_vals[k], f"view {k}")
        assert server.check_whether_all_receive()
        averaged, model_list, idxes = server.aggregate()
        assert idxes == list(range(K))
        assert averaged is model_list[0][1]  # the reference returns client 0's dict, keys rebound
        for k in exp:
            gu.assert_same(averaged[k].cpu(), exp[k], f"round {r} {k}")
        sd = model.state_dict()
        for k in exp:
            if exp[k].dtype == sd[k].dtype:
                gu.assert_same(sd[k].cpu(), exp[k], f"model {k}")
        assert not server.check_whether_all_receive()


def test_resnet50_round(cuda_device):
    """Config 3's state dict (fp32 + int64 counters) through arrival and
    aggregate: all 320 keys bit-exact."""
    K = 4
    raw = host_clients(shapes.resnet50(), K, seed=3, round_idx=5)
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    server = _keyless_server(K, cuda_device)
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert server.bucket is not None and set(server.bucket.groups) == {torch.float32, torch.int64}
    averaged, _, _ = server.aggregate()
    for k in exp:
        assert averaged[k].dtype == exp[k].dtype, k
        gu.assert_same(averaged[k].cpu(), exp[k], k)


def test_plain_dicts_stay_on_the_host(cuda_device):
    """Plain dicts are left where the user put them (:61-62).  FedAvg then
    returns client 0's plain dict, which :90-97 read as a per-client dict
    {client_index: params}: the reference raises KeyError there, and so does
    the mirror, after the reduction itself ran correctly on the host inputs."""
    model = _model().to(cuda_device)
    K = 3
    server = _server(model, K, cuda_device)
    raw = [(n, dict(d)) for n, d in _round(model, K, seed=22, round_idx=0)]
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert server.bucket is None and all(not t.is_cuda for _, d in raw for t in d.values())
    with pytest.raises(KeyError):
        server.aggregate()
    averaged = raw[0][1]  # keys rebound to the average before the KeyError
    for k in exp:
        assert not averaged[k].is_cuda
        gu.assert_same(averaged[k], exp[k], k)


def test_mixed_residency_raises_like_the_reference(cuda_device):
    """One plain (host) dict among moved ones: the reference's `avg += p * w`
    fails on mixed devices with a RuntimeError, and so does this."""
    model = _model().to(cuda_device)
    K = 3
    server = _server(model, K, cuda_device)
    raw = _round(model, K, seed=23, round_idx=0)
    raw[1] = (raw[1][0], dict(raw[1][1]))
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    with pytest.raises(RuntimeError):
        server.aggregate()


def test_other_layout_moves_key_by_key(cuda_device):
    """An update whose layout differs from the first client's is moved key by
    key as in the reference; the result is unchanged."""
    model = _model().to(cuda_device)
    K = 3
    server = _server(model, K, cuda_device)
    raw = _round(model, K, seed=21, round_idx=0)
    extra = OrderedDict(raw[2][1])
    extra["unused.extra"] = torch.ones(3)  # not among client 0's keys: FedAvg ignores it
    raw[2] = (raw[2][0], extra)
    exp = orc.agg(_Args(), copy.deepcopy([(n, OrderedDict((k, v) for k, v in d.items() if k != "unused.extra"))
                                          for n, d in raw]))
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert all(t.is_cuda for t in raw[2][1].values())
    averaged, _, _ = server.aggregate()
    for k in exp:
        gu.assert_same(averaged[k].cpu(), exp[k], k)


def test_same_numel_other_shape_is_not_rebound(cuda_device):
    """The arrival's layout check compares shapes, not element counts: a key
    whose shape differs from the bucket's (same numel) is not rebound to the
    bucket's view (which would reshape the client's tensor); the update moves
    key by key with its own shapes, as the reference moves it."""
    server = _keyless_server(3, cuda_device)
    mk = lambda s: OrderedDict(a=torch.randn(8, 4), b=torch.randn(6))  # noqa: E731
    d0, d1 = mk(0), mk(1)
    server.add_local_trained_result(0, d0, 2)
    server.add_local_trained_result(1, d1, 3)
    assert server.bucket is not None and tuple(d1["a"].shape) == (8, 4)
    d2 = OrderedDict(a=torch.randn(4, 8), b=torch.randn(6))  # transposed shape, same 32 elements
    host_a = d2["a"].clone()
    server.add_local_trained_result(2, d2, 1)
    assert d2["a"].is_cuda and tuple(d2["a"].shape) == (4, 8)
    gu.assert_same(d2["a"].cpu(), host_a, "own shape kept")
    d3 = OrderedDict(a=torch.randn(8, 4).numpy(), b=torch.randn(6))  # not a tensor: never rebound
    assert server._same_layout(d3) is None


def test_int32_key_moves_key_by_key(cuda_device):
    """A dtype the bucket would widen (int32) keeps the reference's per-key move."""
    K = 2
    d0 = OrderedDict(w=torch.randn(5), c=torch.arange(4, dtype=torch.int32))
    d1 = OrderedDict(w=torch.randn(5), c=torch.arange(4, dtype=torch.int32) * 3)
    raw = [(3, d0), (5, d1)]
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    server = _keyless_server(K, cuda_device)
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert server.bucket is None and d0["c"].is_cuda and d0["c"].dtype == torch.int32
    averaged, _, _ = server.aggregate()
    for k in exp:
        gu.assert_same(averaged[k].cpu(), exp[k], k)


class _RoundArgs(_Args):
    dataset = "mnist"
    enable_wandb = False

    def __init__(self, K, comm_round=2, freq=1):
        self.round_idx = 0
        self.comm_round = comm_round
        self.frequency_of_the_test = freq
        self.client_num_per_round = K
        self.client_num_in_total = K


@pytest.mark.parametrize("K", [2, 5])
def test_server_manager_sequence(K, cuda_device):
    """The class swap of INTEGRATION.md §3 inside FedML's real round loop
    (fedml_server_manager.py:174-251, replayed by tests/replay_util.py) for
    two rounds: add xK -> check -> aggregate -> test_on_server_for_all_clients
    -> assess_contribution -> client_selection.  No AttributeError; every
    round's average is bit-exact vs the oracle; the Context holds the round's
    model list and the GPU-evaluated server metrics (acc, loss, None, None)."""
    from replay_util import replay_rounds

    from fedml_amd.context import Context

    Context.reset()
    model = _model().to(cuda_device)
    args = _RoundArgs(K)
    g = torch.Generator().manual_seed(5)
    test_set = torch.utils.data.TensorDataset(torch.randn(40, 37, generator=g), torch.randint(0, 3, (40,), generator=g))
    loader = torch.utils.data.DataLoader(test_set, batch_size=16)
    server = FedMLAggregator(None, loader, 0, {}, {}, {}, K, cuda_device, args, MI355XServerAggregator(model, args))
    expected = {}

    def updates(r):
        raw = _round(model, K, seed=70 + r, round_idx=r)
        for _, d in raw:  # a variance the evaluation can take the root of
            d["1.running_var"].abs_()
        expected[r] = orc.agg(_Args(), copy.deepcopy(raw))
        return raw

    out = replay_rounds(server, args, list(range(1, K + 1)), updates, rounds=2)
    for o in out:
        for k, e in expected[o["round_idx"]].items():
            gu.assert_same(o["global"][k].cpu(), e, f"round {o['round_idx']} {k}")
        assert o["ctx_model_list"] is o["model_list"]
        acc, loss, a, b = o["metrics"]
        assert a is None and b is None and 0.0 <= acc <= 1.0 and loss > 0
    assert out[1]["metrics_last"] == out[0]["metrics"]
    # round 1's metrics are those of the model holding round 1's average
    with torch.no_grad():
        x, y = test_set.tensors
        pred = model(x.to(cuda_device)).argmax(1).cpu()
    assert out[1]["metrics"][0] == (pred == y).sum().item() / len(y)


def _ingested(K, device, seed=21, entries=None):
    entries = entries or cases_entries()
    raw = host_clients(entries, K, seed=seed, round_idx=2)
    host = copy.deepcopy(raw)
    server = _keyless_server(K, device)
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    return server, raw, host


def cases_entries():
    return [("w", (300, 17), torch.float32), ("b", (17,), torch.float32), ("h", (77,), torch.bfloat16),
            ("n", (), torch.int64), ("z", (0,), torch.float32)]


def test_aggregate_reduces_the_resident_rows(cuda_device, monkeypatch):
    """aggregate() over the ingested dicts reduces the bucket rows directly
    (agg_operator._reduce_resident: no walk over K x keys views), bit-exact."""
    from fedml_amd import agg_operator as ao

    def no_walk(*a, **k):
        raise AssertionError("the resident round walked the views")

    server, raw, host = _ingested(6, cuda_device)
    exp = orc.agg(_Args(), copy.deepcopy(host))
    monkeypatch.setattr(ao, "_reduce_device_walked", no_walk)
    averaged, _, _ = server.aggregate()
    for k in exp:
        assert averaged[k].dtype == exp[k].dtype, k
        gu.assert_same(averaged[k].cpu(), exp[k], k)


def test_resident_rounds_in_any_order_and_subset(cuda_device):
    """agg() over the ingested dicts in another order, or a subset of them:
    the rows go in the list's order (a pointer table per slot list)."""
    from fedml_amd.agg_operator import FedMLAggOperator

    server, raw, host = _ingested(7, cuda_device, seed=22)
    for order in ([6, 2, 0, 5, 1, 4, 3], [3, 1, 5], [4]):
        lst = [(server.sample_num_dict[i], server.model_dict[i]) for i in order]
        exp = orc.agg(_Args(), [copy.deepcopy(host[i]) for i in order])
        keep = {k: t for k, t in lst[0][1].items()}
        res = FedMLAggOperator.agg(_Args(), lst)
        assert res is lst[0][1]
        for k in exp:
            gu.assert_same(res[k].cpu(), exp[k], f"{order} {k}")
        for k, t in keep.items():  # the next order starts from the views again
            lst[0][1][k] = t


def test_a_dict_changed_after_ingest_is_walked(cuda_device, monkeypatch):
    """A hook that rebinds one value of one client (a defense scaling an
    update) makes the round leave the rows alone: the walked path reduces
    what the dicts hold now."""
    from fedml_amd import agg_operator as ao

    server, raw, host = _ingested(5, cuda_device, seed=23)
    server.model_dict[3]["w"] = server.model_dict[3]["w"] * 2.0
    host[3][1]["w"] = host[3][1]["w"] * 2.0
    walked = []
    real = ao._reduce_device_walked
    monkeypatch.setattr(ao, "_reduce_device_walked", lambda *a: walked.append(1) or real(*a))
    exp = orc.agg(_Args(), copy.deepcopy(host))
    averaged, _, _ = server.aggregate()
    assert walked
    for k in exp:
        gu.assert_same(averaged[k].cpu(), exp[k], k)
