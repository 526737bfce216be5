"""The in-process multi-device bucket (fedml_amd.multidev) on the GPU: G
shards placed on the box's one MI355X (each its own ClientBucket, copy stream,
staging and pinned results), so the slicing, the per-shard streams and the
reassembly run exactly as on G GPUs.  Bit-exact against the oracle and the
reference's golden vectors."""
from __future__ import annotations

import copy
from collections import OrderedDict

import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import agg_operator as ao
from fedml_amd import shapes
from fedml_amd.bucket import ClientBucket
from fedml_amd.cross_silo import FedMLAggregator
from fedml_amd.multidev import MultiDeviceBucket
from fedml_amd.server_aggregator import MI355XServerAggregator
from fedml_amd.synth import host_clients
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu

ENTRIES = cases._entries(cases.RESNET_MINI) + [
    ("x.big", (70001,), torch.float32), ("x.empty", (0,), torch.float32), ("x.scalar", (), torch.float32),
    ("x.odd", (1023,), torch.float32), ("x.count", (), torch.int64)]
ENTRIES_BF16 = [(k, s, torch.bfloat16 if d == torch.float32 else d) for k, s, d in ENTRIES]


class _Args:
    federated_optimizer = "FedAvg"


@pytest.mark.parametrize("G", [1, 2, 4])
@pytest.mark.parametrize("entries", [ENTRIES, ENTRIES_BF16], ids=["f32", "bf16"])
def test_bucket_round_trip_matches_oracle(G, entries, cuda_device):
    K = 9
    raw = host_clients(entries, K, seed=40 + G, round_idx=3)
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    b = MultiDeviceBucket(entries, K, [cuda_device] * G)
    assert len(b.shards) == G
    for i, (n, d) in enumerate(raw):
        b.put(i, d, n)
    ns = [n for n, _ in raw]
    host = b.reduce_to_host(b.weights(ns))
    assert list(host) == list(exp)
    for k, e in exp.items():
        assert not host[k].is_cuda and host[k].dtype == e.dtype
        gu.assert_same(host[k], e, f"G={G} host {k}")
    dev = b.aggregate(ns)
    for k, e in exp.items():
        assert dev[k].is_cuda
        gu.assert_same(dev[k].cpu(), e, f"G={G} device {k}")
    # a second round on the same slots, results independent of the first
    raw2 = host_clients(entries, K, seed=90 + G, round_idx=4)
    exp2 = orc.agg(_Args(), copy.deepcopy(raw2))
    for i, (n, d) in enumerate(raw2):
        b.put(i, d, n)
    host2 = b.reduce_to_host(b.weights([n for n, _ in raw2]))
    for k in exp:
        gu.assert_same(host2[k], exp2[k], f"round 2 {k}")
        gu.assert_same(host[k], exp[k], f"round 1 kept {k}")


def test_shards_use_their_own_streams(cuda_device):
    """Every shard stages and copies on its own copy stream and D2H stream,
    as it would on its own GPU."""
    K = 3
    raw = host_clients(ENTRIES, K, seed=7)
    b = MultiDeviceBucket(ENTRIES, K, [cuda_device] * 3)
    for i, (n, d) in enumerate(raw):
        b.put(i, d, n)
    b.reduce_to_host(b.weights([n for n, _ in raw]))
    copies = [s._copy for s in b.shards]
    d2hs = [s._d2h for s in b.shards]
    assert all(c is not None for c in copies) and len({id(c) for c in copies}) == 3
    assert all(c is not None for c in d2hs) and len({id(c) for c in d2hs}) == 3


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("name", ["ragged_f32_k128", "kat_fake_model_list_k10", "cfg2_cnn_web_k32", "ragged_bf16_k32"])
def test_agg_with_fedagg_devices_matches_reference(G, name, cuda_device):
    """FedMLAggOperator.agg on host dicts with args.fedagg_devices listing G
    devices: the round goes through a MultiDeviceBucket (one batched pack per
    shard) and matches the reference's golden vectors bit for bit."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    args = cases.Args(spec)
    args.fedagg_devices = [cuda_device] * G
    ao._MULTI.clear()
    res = ao.FedMLAggOperator.agg(args, raw)
    gu.assert_groups(res, meta, arrays, name)
    assert len(ao._MULTI) == 1
    b = next(iter(ao._MULTI.values()))
    assert 1 <= len(b.shards) <= G


def test_one_listed_device_after_a_multi_device_round(cuda_device):
    """A round with args.fedagg_devices naming ONE device after a multi-device
    round of the same layout runs on that device and drops the cached
    multi-device bucket (it does not reuse the earlier placement)."""
    meta, arrays = gu.load("ragged_f32_k17")
    spec = meta["spec"]
    args = cases.Args(spec)
    args.fedagg_devices = [cuda_device] * 2
    ao._MULTI.clear()
    ao._BUCKETS.clear()
    gu.assert_groups(ao.FedMLAggOperator.agg(args, cases.build_inputs(spec)), meta, arrays, "multi")
    assert len(ao._MULTI) == 1
    args.fedagg_devices = [cuda_device]
    gu.assert_groups(ao.FedMLAggOperator.agg(args, cases.build_inputs(spec)), meta, arrays, "one")
    assert len(ao._MULTI) == 0 and len(ao._BUCKETS) == 1


@pytest.mark.parametrize("G", [2, 3])
def test_agg_multidevice_per_client_staging(G, cuda_device, monkeypatch):
    """Rounds above the batched-pack size go client by client through each
    shard's staging ring (put_from_tables): forced here on config 3's
    ResNet-50 state dict (320 keys, int64 counters) at K = 3."""
    monkeypatch.setattr(ao, "_BATCH_MAX_BYTES", 0)
    K = 3
    raw = host_clients(shapes.resnet50(), K, seed=8, round_idx=2)
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    args = _Args()
    args.fedagg_devices = ",".join(["0"] * G)
    ao._MULTI.clear()
    res = ao.FedMLAggOperator.agg(args, raw)
    assert len(ao._MULTI) == 1
    for k, e in exp.items():
        assert res[k].dtype == e.dtype
        gu.assert_same(res[k], e, k)


@pytest.mark.parametrize("G", [2, 3])
def test_cross_silo_multidevice_round_reduces_resident_rows(G, cuda_device, monkeypatch):
    """The multi-device cross-silo round end reduces every shard's rows in
    place (agg_operator._reduce_resident on a MultiDeviceBucket), in any
    client order, bit-exact; a rebound value sends the round to the walk."""
    def no_walk(*a, **k):
        raise AssertionError("walked")

    args = _Args()
    args.fedagg_devices = [cuda_device] * G
    K = 6
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, cuda_device, args,
                             MI355XServerAggregator(torch.nn.Linear(1, 1), args))
    server.aggregator.set_model_params = lambda p: None
    raw = host_clients(ENTRIES, K, seed=61, round_idx=1)
    host = copy.deepcopy(raw)
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert isinstance(server.bucket, MultiDeviceBucket)
    real = ao._reduce_device_walked
    monkeypatch.setattr(ao, "_reduce_device_walked", no_walk)
    order = [4, 0, 5, 2, 1, 3]
    lst = [(server.sample_num_dict[i], server.model_dict[i]) for i in order]
    keep = dict(lst[0][1])
    res = ao.FedMLAggOperator.agg(_Args(), lst)
    exp = orc.agg(_Args(), [copy.deepcopy(host[i]) for i in order])
    for k, e in exp.items():
        gu.assert_same(res[k].cpu(), e, k)
    lst[0][1].update(keep)  # back to the views
    monkeypatch.setattr(ao, "_reduce_device_walked", real)
    server.model_dict[2]["x.big"] = server.model_dict[2]["x.big"] + 1.0
    host[2][1]["x.big"] = host[2][1]["x.big"] + 1.0
    res = ao.FedMLAggOperator.agg(_Args(), [(server.sample_num_dict[i], server.model_dict[i]) for i in range(K)])
    exp = orc.agg(_Args(), copy.deepcopy(host))
    for k, e in exp.items():
        gu.assert_same(res[k].cpu(), e, k)


@pytest.mark.parametrize("G", [2, 4])
def test_cross_silo_rounds_on_several_shards(G, cuda_device):
    """The cross-silo mirror with args.fedagg_devices: updates land in a
    MultiDeviceBucket on arrival, the dicts hold one-device views of their
    slots (values and dtypes of the update), and aggregate() (the plugin
    path, agg() on those views) is bit-exact over two rounds."""
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.BatchNorm1d(19), torch.nn.Linear(19, 3)).to(cuda_device)
    args = _Args()
    args.fedagg_devices = [cuda_device] * G
    K = 5
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, cuda_device, args, MI355XServerAggregator(model, args))
    entries = [(k, tuple(t.shape), t.dtype) for k, t in model.state_dict().items()]
    for r in range(2):
        raw = host_clients(entries, K, seed=30 + r, round_idx=r)
        exp = orc.agg(_Args(), copy.deepcopy(raw))
        for i, (n, d) in enumerate(raw):
            vals = OrderedDict((k, t.clone()) for k, t in d.items())
            server.add_local_trained_result(i, d, n)
            for k, t in d.items():
                assert t.is_cuda and t.dtype == vals[k].dtype
                gu.assert_same(t.cpu(), vals[k], f"view {k}")
        assert isinstance(server.bucket, MultiDeviceBucket) and len(server.bucket.shards) == G
        assert server.check_whether_all_receive()
        averaged, model_list, _ = server.aggregate()
        for k, e in exp.items():
            gu.assert_same(averaged[k].cpu(), e, f"round {r} {k}")
        sd = model.state_dict()
        for k, e in exp.items():
            if e.dtype == sd[k].dtype:
                gu.assert_same(sd[k].cpu(), e, f"model {k}")


def test_device_walk_groups_keys_by_device(cuda_device):
    """agg() on device dicts whose keys sit in different buckets (the views of
    a MultiDeviceBucket): the native walker groups the keys by device and the
    pipelined launches reduce every key; equal to a one-bucket round."""
    K = 6
    raw = host_clients(shapes.resnet50()[:40], K, seed=12)
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    b = MultiDeviceBucket([(k, tuple(t.shape), t.dtype) for k, t in raw[0][1].items()], K, [cuda_device] * 4,
                          promote_ints=False)
    views = []
    for i, (n, d) in enumerate(raw):
        b.put(i, d, n)
        views.append((n, b.view(i)))
    b.sync_ingest()
    w = ao._walker()
    groups = w.group_by_device(views[0][1], list(views[0][1]))
    assert [g for g, _ in groups] == [cuda_device.index]
    assert sorted(i for _, idx in groups for i in idx) == list(range(len(views[0][1])))
    res = ao.FedMLAggOperator.agg(_Args(), views)
    for k, e in exp.items():
        gu.assert_same(res[k].cpu(), e, k)
    single = ClientBucket([(k, tuple(t.shape), t.dtype) for k, t in raw[0][1].items()], K, cuda_device)
    assert single.num_elements() == b.num_elements()


def _over_hbm_node(monkeypatch, cuda_device, G: int = 4):
    """A node of G GPUs (all mapped onto the box's one MI355X) whose default
    device has 1 KB of HBM free: every round above that "exceeds one GPU"."""
    from fedml_amd import multidev

    monkeypatch.setattr(torch.cuda, "device_count", lambda: G)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d=None: (1 << 10, 288 << 30))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda d=None: 0)
    monkeypatch.setattr(multidev, "visible_devices", lambda: [cuda_device] * G)


@pytest.mark.parametrize("name", ["ragged_f32_k128", "ragged_bf16_k32", "cfg2_cnn_web_k32"])
def test_agg_spreads_an_over_hbm_round_unprompted(name, cuda_device, monkeypatch):
    """north_star's trigger end to end: no fedagg_devices, but the round does
    not fit the default GPU's free HBM, so FedMLAggOperator.agg builds a
    MultiDeviceBucket over the visible GPUs by itself, and the result matches
    the reference's golden vectors bit for bit.  A second round of the same
    layout reuses that bucket (placement decided once)."""
    _over_hbm_node(monkeypatch, cuda_device)
    monkeypatch.setattr(ao, "_HOST_ROUND_MAX_BYTES", 0)  # small rounds would otherwise take the one-call path
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    ao._MULTI.clear()
    ao._BUCKETS.clear()
    res = ao.FedMLAggOperator.agg(cases.Args(spec), cases.build_inputs(spec))
    gu.assert_groups(res, meta, arrays, name)
    assert len(ao._MULTI) == 1 and not ao._BUCKETS
    b = next(iter(ao._MULTI.values()))
    assert isinstance(b, MultiDeviceBucket) and len(b.shards) >= 2
    res = ao.FedMLAggOperator.agg(cases.Args(spec), cases.build_inputs(spec))
    gu.assert_groups(res, meta, arrays, name + " (round 2)")
    assert len(ao._MULTI) == 1 and next(iter(ao._MULTI.values())) is b
    ao._MULTI.clear()


def test_cross_silo_spreads_an_over_hbm_round_unprompted(cuda_device, monkeypatch):
    """The cross-silo mirror's first update decides the placement: with the
    round over the free HBM and 4 GPUs visible it builds a 4-shard
    MultiDeviceBucket without fedagg_devices; aggregate() is bit-exact."""
    _over_hbm_node(monkeypatch, cuda_device)
    torch.manual_seed(1)
    model = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.BatchNorm1d(19), torch.nn.Linear(19, 3)).to(cuda_device)
    args = _Args()
    K = 5
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, cuda_device, args, MI355XServerAggregator(model, args))
    entries = [(k, tuple(t.shape), t.dtype) for k, t in model.state_dict().items()]
    raw = host_clients(entries, K, seed=77, round_idx=1)
    exp = orc.agg(_Args(), copy.deepcopy(raw))
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert isinstance(server.bucket, MultiDeviceBucket) and len(server.bucket.shards) == 4
    assert server.check_whether_all_receive()
    averaged, _, _ = server.aggregate()
    for k, e in exp.items():
        gu.assert_same(averaged[k].cpu(), e, k)
