"""FedOpt over several GPUs of one server process (MultiDeviceFedOptServer):
whole keys per device, each device its own fused server step.  Every case is
checked bit for bit against the one-device FedOptServer (itself pinned to the
reference's FedOptAggregator / FedOptAPI golden vectors in test_gpu_fedopt.py),
parameters, buffers and optimizer state alike, with all G shards on the box's
one MI355X."""
from __future__ import annotations

from collections import OrderedDict

import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import multidev
from fedml_amd.fedopt import FedOptServer, MultiDeviceFedOptServer, make_fedopt_server
from fedml_amd.synth import host_clients

pytestmark = pytest.mark.gpu

ALL_CASES = (cases.FEDOPT_CASES + cases.FEDOPT_ADAM_CASES + cases.FEDOPT_ADAGRAD_CASES
             + cases.FEDOPT_RMSPROP_CASES + cases.FEDOPT_ADAMW_CASES)


def _opt(spec):
    return spec.get("optimizer", "adam" if spec in cases.FEDOPT_ADAM_CASES else "sgd")


def _run_round(server, raw):
    for i, (n, d) in enumerate(raw):
        server.add_local_trained_result(i, d, n)
    assert server.check_whether_all_receive()
    return OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items())


def _same_state(a, b, what):
    assert a.keys() == b.keys(), what
    assert a["step"] == b["step"], what
    for name in a:
        if name == "step":
            continue
        assert list(a[name]) == list(b[name]), f"{what} {name} key order"
        for k in a[name]:
            gu.assert_same(a[name][k].cpu(), b[name][k].cpu(), f"{what} {name} {k}")


@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("spec", ALL_CASES, ids=lambda s: s["name"])
def test_multi_device_fedopt_equals_one_device(spec, G, cuda_device):
    opt = _opt(spec)
    init = cases.fedopt_global_init(spec)
    one = FedOptServer(init, cases.FEDOPT_PARAMS, spec["K"], opt, spec["lr"], spec.get("momentum", 0.0), cuda_device)
    multi = MultiDeviceFedOptServer(init, one.param_names, spec["K"], opt, spec["lr"], spec.get("momentum", 0.0),
                                    [cuda_device] * G)
    assert len(multi.servers) >= 2
    owners = [{k for k, _, _ in s.bucket.entries} for s in multi.servers]
    assert sum(len(o) for o in owners) == len(init) and set().union(*owners) == set(init)
    _same_state(one.optimizer_state(), multi.optimizer_state(), f"{spec['name']} before round 0")
    gsd = init
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        a = _run_round(one, raw)
        b = _run_round(multi, cases.fedopt_round_inputs(spec, gsd, r))
        assert list(a) == list(b)
        for k in a:
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
            gu.assert_same(b[k], a[k], f"{spec['name']} G={G} round {r} {k}")
        _same_state(one.optimizer_state(), multi.optimizer_state(), f"{spec['name']} round {r}")
        gsd = a
    # the same bytes up to the 256-B row alignment each device's layout pads
    assert abs(multi.algorithmic_bytes() - one.algorithmic_bytes()) <= 0.05 * one.algorithmic_bytes() + 4096


@pytest.mark.parametrize("opt", ["sgd", "adam", "adagrad", "rmsprop", "adamw"])
def test_multi_device_optimizer_state_resume(opt, cuda_device):
    """A multi-device server resumed from a one-device server's state (and the
    other way round) continues bit-identically: the state is keyed by
    parameter name, not by device."""
    entries = [("a.weight", (33, 70), torch.float32), ("a.bias", (33,), torch.float32),
               ("bn.running_mean", (33,), torch.float32), ("b.weight", (5, 33), torch.float32),
               ("bn.num_batches_tracked", (), torch.int64)]
    params = ["a.weight", "a.bias", "b.weight"]
    K = 4
    init = host_clients(entries, 1, seed=11)[0][1]
    mom = 0.9 if opt == "sgd" else 0.0
    one = FedOptServer(init, params, K, opt, 0.05, mom, cuda_device)
    gsd = init
    for r in range(2):
        gsd = _run_round(one, host_clients(entries, K, seed=30 + r, round_idx=r))
    multi = MultiDeviceFedOptServer(gsd, params, K, opt, 0.05, mom, [cuda_device] * 3)
    multi.load_optimizer_state(one.optimizer_state())
    _same_state(one.optimizer_state(), multi.optimizer_state(), f"{opt} resumed")
    back = FedOptServer(gsd, params, K, opt, 0.05, mom, cuda_device)
    raw = host_clients(entries, K, seed=40, round_idx=2)
    a = _run_round(one, raw)
    b = _run_round(multi, host_clients(entries, K, seed=40, round_idx=2))
    for k in a:
        gu.assert_same(b[k], a[k], f"{opt} {k}")
    back.load_optimizer_state(multi.optimizer_state())
    _same_state(one.optimizer_state(), back.optimizer_state(), f"{opt} back to one device")


def test_device_resident_updates(cuda_device):
    """Client updates already on the GPU go in by D2D copies; mixed host and
    device keys of one client are fine."""
    entries = [("w", (1000, 37), torch.float32), ("b", (1000,), torch.float32), ("v", (77, 5), torch.float32)]
    K = 5
    init = host_clients(entries, 1, seed=2)[0][1]
    one = FedOptServer(init, ["w", "b", "v"], K, "sgd", 1.0, 0.9, cuda_device)
    multi = MultiDeviceFedOptServer(init, ["w", "b", "v"], K, "sgd", 1.0, 0.9, [cuda_device] * 2)
    for r in range(2):
        raw = host_clients(entries, K, seed=60 + r, round_idx=r)
        mixed = [(n, OrderedDict((k, t.to(cuda_device) if k != "b" else t) for k, t in d.items())) for n, d in raw]
        a = _run_round(one, raw)
        b = _run_round(multi, mixed)
        for k in a:
            gu.assert_same(b[k], a[k], f"round {r} {k}")


class _Args:
    pass


def test_factory_places_the_server(cuda_device, monkeypatch):
    """make_fedopt_server: one device by default; args.fedagg_devices lists
    the GPUs; an over-HBM round on a multi-GPU node spreads by itself."""
    entries = [("w", (300, 64), torch.float32), ("b", (300,), torch.float32), ("u", (64, 9), torch.float32)]
    init = host_clients(entries, 1, seed=3)[0][1]
    s = make_fedopt_server(init, ["w", "b", "u"], 4, "adam", 0.01, device=cuda_device)
    assert isinstance(s, FedOptServer)
    args = _Args()
    args.fedagg_devices = [str(cuda_device)] * 2
    s = make_fedopt_server(init, ["w", "b", "u"], 4, "adam", 0.01, device=cuda_device, args=args)
    assert isinstance(s, MultiDeviceFedOptServer) and len(s.servers) == 2
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d=None: (1 << 10, 288 << 30))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda d=None: 0)
    monkeypatch.setattr(multidev, "visible_devices", lambda: [cuda_device] * 4)
    s = make_fedopt_server(init, ["w", "b", "u"], 4, "adam", 0.01, device=cuda_device, args=_Args())
    assert isinstance(s, MultiDeviceFedOptServer) and len(s.servers) == 3  # three keys, three devices used
    one = FedOptServer(init, ["w", "b", "u"], 4, "adam", 0.01, cuda_device)
    raw = host_clients(entries, 4, seed=9)
    a, b = _run_round(one, raw), _run_round(s, host_clients(entries, 4, seed=9))
    for k in a:
        gu.assert_same(b[k], a[k], k)


def test_multi_device_server_exposes_the_server_settings(cuda_device):
    """The multi-device server carries FedOptServer's scalar settings and names
    its per-shard buckets and devices."""
    entries = [("w", (300, 64), torch.float32), ("b", (300,), torch.float32)]
    init = host_clients(entries, 1, seed=5)[0][1]
    one = FedOptServer(init, ["w", "b"], 3, "sgd", 0.5, 0.9, cuda_device)
    multi = MultiDeviceFedOptServer(init, ["w", "b"], 3, "sgd", 0.5, 0.9, [cuda_device] * 2)
    for a in ("optimizer", "lr", "momentum", "betas", "eps", "alpha", "weight_decay", "lr_decay", "worker_num",
              "param_names"):
        assert getattr(multi, a) == getattr(one, a), a
    assert multi.device == one.device and multi.bucket is multi.buckets[0]
    assert len(multi.buckets) == len(multi.devices) == 2
