"""Random rounds through the drop-in against the oracle, on the GPU.

Each case draws the optimizer branch (FedAvg, FedProx, FedAvg_seq, FedDyn),
the client count (1 to 600), a handful of keys with random dtypes (f32, bf16,
f16, f64, int64, int32, uint8, bool) and lengths around every tile-shape
threshold of the dispatch (tiny / narrow / small / mid / wide tiles, 0, 1 and
ragged tails), host or device residency, the accumulation mode, and now and
then NaN / inf / -0.0 / denormal values.  FedMLAggOperator.agg must return
the oracle's bits (agg_operator.py:33-63 restated in oracle/fedavg_oracle.py,
pinned to the reference's fixtures), client 0's dict rebinding included.
The same for the MPI simulation's term order (orc.mpi_fedavg) and for the
SCAFFOLD / Mime 3-tuples, client 0's in-place control variates included,
and for three-round FedOptServer runs (five fused optimizers, parameter keys
interleaved with buffer keys), optimizer state included, and for
three-round runs of the cross-silo mirror (arrival order, odd updates, the
server model on the host or the GPU), and for defended rounds (median,
trimmed mean, Krum / multi-Krum, norm-diff clipping), and with the round
spread over 2-4 shards (args.fedagg_devices), and with non-contiguous,
unaligned and nn.Parameter client tensors, and ClientBucket rounds fed by
put / device put / FAGG messages.
Seeded: a failure names its case and replays.
"""
from __future__ import annotations

import copy
import os
import random
from collections import OrderedDict

import numpy as np
import pytest
import torch

import golden_util as gu
from fedml_amd.agg_operator import FedMLAggOperator
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu

_LENGTHS = [0, 1, 3, 31, 255, 256, 1023, 1024, 4095, 4096, 4097, 16383, 32767, 32768, 70001, 262_147,
            (1 << 20) - 1, (1 << 20) + 3]
_WEIGHTED = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32, torch.uint8,
             torch.bool]
_SUMMED = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64]
# FEDAGG_FUZZ_SCALE=n multiplies every case count (a longer campaign; new seeds come after the defaults)
_SCALE = max(1, int(os.environ.get("FEDAGG_FUZZ_SCALE", "1")))
# FEDAGG_FUZZ_SEED0=s starts every seed range at s (a campaign over fresh seeds)
_SEED0 = int(os.environ.get("FEDAGG_FUZZ_SEED0", "0"))
_CASES = 160 * _SCALE
_CASES_3 = 120 * _SCALE  # MPI order, SCAFFOLD / Mime tuples
_ELEMS_PER_CASE = 24 << 20  # K x elements, so the oracle's numpy loop stays short


class _Args:
    def __init__(self, opt, acc):
        self.federated_optimizer = opt
        if acc:
            self.fedagg_low_precision_acc = acc


def _values(rnd: random.Random, g: torch.Generator, n: int, dt: torch.dtype, special: bool) -> torch.Tensor:
    if dt == torch.bool:
        return torch.randint(0, 2, (n,), generator=g).bool()
    if dt == torch.uint8:
        return torch.randint(0, 256, (n,), generator=g).to(torch.uint8)
    if dt in (torch.int64, torch.int32):
        return torch.randint(-100, 100, (n,), generator=g).to(dt)
    t = (torch.randn(n, generator=g, dtype=torch.float64) * 0.05).to(dt)
    if special and n:
        picks = torch.randint(0, n, (min(n, 8),), generator=g)
        vals = [float("nan"), float("inf"), -float("inf"), -0.0, 1e-40, -1e-42, 3e38]
        for j, p in enumerate(picks.tolist()):
            t[p] = vals[j % len(vals)]
    return t


def _case(seed: int):
    rnd = random.Random(seed)
    g = torch.Generator().manual_seed(seed)
    opt = rnd.choice(["FedAvg"] * 6 + ["FedProx", "FedAvg_seq", "FedDyn"])
    summed = opt in ("FedAvg_seq", "FedDyn")
    K = rnd.choice([1, 2, 3, 5, 8, 16, 31, 48, 64, 128, 129, 256, 300, 513, 600])
    nkeys = rnd.randint(1, 5)
    keys = []
    budget = _ELEMS_PER_CASE // K
    for j in range(nkeys):
        dt = rnd.choice(_SUMMED if summed else _WEIGHTED)
        n = rnd.choice([x for x in _LENGTHS if x <= budget] or [1])
        budget = max(1, budget - n)
        shape = (n,) if n < 4 or rnd.random() < 0.5 else (n // 2, 2) if n % 2 == 0 else (n,)
        keys.append((f"k{j}", shape, dt))
    special = rnd.random() < 0.15
    raw = []
    for i in range(K):
        d = OrderedDict((k, _values(rnd, g, int(np.prod(s)), dt, special).reshape(s)) for k, s, dt in keys)
        n_i = rnd.choice([1, 7, 100, 1000, 3.5, 10 ** 12])
        raw.append((n_i, d))
    acc = rnd.choice([None, None, None, "fp32"]) if not summed else None
    device = rnd.random() < 0.5
    return opt, K, keys, raw, acc, device


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + _CASES)))
def test_random_round_matches_the_oracle(seed, cuda_device):
    opt, K, keys, raw, acc, device = _case(seed)
    what = f"seed {seed}: {opt} K={K} acc={acc} device={device} keys={[(k, s, str(d)) for k, s, d in keys]}"
    host = copy.deepcopy(raw)
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    got = FedMLAggOperator.agg(_Args(opt, acc), raw)
    exp_src = copy.deepcopy(host)
    exp = orc.agg(_Args(opt, None), exp_src)
    assert list(got) == list(exp), what
    ws = [n / sum(n for n, _ in host) for n, _ in host]
    for k, s, dt in keys:
        e = exp[k]
        if acc == "fp32" and dt in (torch.bfloat16, torch.float16):
            e = orc.wsum_acc32([d[k] for _, d in host], ws)
        a = got[k]
        assert a.is_cuda == device, what
        gu.assert_same(a.cpu(), e, f"{what} key {k}")
    assert got is raw[0][1], what  # client 0's dict, keys rebound (agg_operator.py:36-44)


_MPI_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64]


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + _CASES_3)))
def test_random_mpi_round_matches_the_oracle(seed, cuda_device):
    """The MPI simulation's term order (FedAVGAggregator.py:99-116) through
    fedml_amd.simulation.fedavg_mpi_aggregate, random shapes, dtypes, sample
    counts (integers, floats, 10^15: int64 products wrap) and residency."""
    from fedml_amd.simulation import fedavg_mpi_aggregate

    rnd = random.Random(1000 + seed)
    g = torch.Generator().manual_seed(1000 + seed)
    K = rnd.choice([1, 2, 5, 17, 64, 130, 300])
    budget = _ELEMS_PER_CASE // 2 // K
    keys = []
    for j in range(rnd.randint(1, 4)):
        n = rnd.choice([x for x in _LENGTHS if x <= budget] or [1])
        budget = max(1, budget - n)
        keys.append((f"k{j}", (n,), rnd.choice(_MPI_DTYPES)))
    special = rnd.random() < 0.15
    raw = [(rnd.choice([1, 3, 250, 10 ** 15, 2.5, 7.25]),
            OrderedDict((k, _values(rnd, g, s[0], dt, special)) for k, s, dt in keys)) for _ in range(K)]
    device = rnd.random() < 0.5
    what = f"mpi seed {seed}: K={K} device={device} keys={[(k, s, str(d)) for k, s, d in keys]}"
    host = copy.deepcopy(raw)
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    got = fedavg_mpi_aggregate(raw)
    exp = orc.mpi_fedavg(host)
    assert list(got) == list(exp), what
    for k in exp:
        gu.assert_same(got[k].cpu(), exp[k], f"{what} key {k}")


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + _CASES_3)))
def test_random_scaffold_mime_round_matches_the_oracle(seed, cuda_device):
    """SCAFFOLD and Mime (3-tuples, agg_operator.py:100-133) on the real
    kernels: random dtypes and lengths, host or device, both results and the
    in-place update of client 0's control-variate tensors (SCAFFOLD)."""
    rnd = random.Random(2000 + seed)
    g = torch.Generator().manual_seed(2000 + seed)
    opt = rnd.choice(["SCAFFOLD", "Mime"])
    K = rnd.choice([1, 2, 3, 8, 33, 130])
    budget = _ELEMS_PER_CASE // 4 // K
    keys = []
    for j in range(rnd.randint(1, 4)):
        n = rnd.choice([x for x in _LENGTHS if x <= budget] or [1])
        budget = max(1, budget - n)
        keys.append((f"k{j}", (n,), rnd.choice([torch.float32, torch.bfloat16, torch.float64, torch.int64])))
    mk = lambda: OrderedDict((k, _values(rnd, g, s[0], dt, False)) for k, s, dt in keys)  # noqa: E731
    raw = [(rnd.choice([1, 4, 9, 2.5]), mk(), mk()) for _ in range(K)]
    device = rnd.random() < 0.5
    what = f"{opt} seed {seed}: K={K} device={device} keys={[(k, s, str(d)) for k, s, d in keys]}"
    host = copy.deepcopy(raw)
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in a.items()),
                OrderedDict((k, t.to(cuda_device)) for k, t in b.items())) for n, a, b in raw]
    c0_got, c0_exp = list(raw[0][2].values()), list(host[0][2].values())
    args = _Args(opt, None)
    args.client_num_per_round = K
    args.client_num_in_total = 4 * K
    got = FedMLAggOperator.agg(args, raw)
    exp = orc.agg(args, host)
    assert isinstance(got, tuple) and len(got) == len(exp), what
    for gd, ed in zip(got, exp):
        assert list(gd) == list(ed), what
        for k in ed:
            gu.assert_same(gd[k].cpu(), ed[k], f"{what} key {k}")
    for j, (a, e) in enumerate(zip(c0_got, c0_exp)):  # client 0's own tensors (SCAFFOLD `+=` into them)
        gu.assert_same(a.cpu(), e, f"{what} client-0 tensor {j}")


_FEDOPT = [("sgd", 0.0), ("sgd", 0.9), ("adam", 0.0), ("adamw", 0.0), ("adagrad", 0.0), ("rmsprop", 0.0),
           ("adamax", 0.0), ("nadam", 0.0), ("radam", 0.0), ("adadelta", 0.0), ("asgd", 0.0), ("rprop", 0.0)]


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 60 * _SCALE)))
def test_random_fedopt_rounds_match_the_oracle(seed, cuda_device):
    """FedOptServer (FedOptAggregator.py:81-125, fedopt_api.py:121-130) over
    three rounds: a random optimizer, learning rate and client count, fp32
    parameter keys interleaved with fp32 / bf16 / int64 buffer keys (so the
    fused runs split at random places), random sample counts.  Parameters,
    buffers and optimizer state bit-exact against the oracle (IEEE sqrt)."""
    from fedml_amd.fedopt import FedOptServer

    rnd = random.Random(3000 + seed)
    g = torch.Generator().manual_seed(3000 + seed)
    opt, mom = rnd.choice(_FEDOPT)
    lr = rnd.choice([1.0, 0.5, 0.1, 0.01, 3e-4])
    K = rnd.choice([1, 2, 3, 7, 16, 40, 129])
    budget = (8 << 20) // K
    entries, names = [], []
    for j in range(rnd.randint(1, 6)):
        n = rnd.choice([x for x in _LENGTHS if 0 < x <= budget] or [1])
        budget = max(1, budget - n)
        kind = rnd.choice(["p", "p", "p", "f32", "bf16", "i64"])
        dt = {"p": torch.float32, "f32": torch.float32, "bf16": torch.bfloat16, "i64": torch.int64}[kind]
        entries.append((f"k{j}", n, dt))
        if kind == "p":
            names.append(f"k{j}")
    init = OrderedDict((k, _values(rnd, g, n, dt, False)) for k, n, dt in entries)
    what = f"fedopt seed {seed}: {opt} m={mom} lr={lr} K={K} keys={[(k, n, str(d), k in names) for k, n, d in entries]}"
    srv = FedOptServer(init, names, K, opt, lr, mom, cuda_device)
    prev, state = init, {}
    for r in range(3):
        raw = [(rnd.choice([1, 5, 64, 2.5]), OrderedDict(
            (k, (t + _values(rnd, g, t.numel(), t.dtype, False) * 0.1).to(t.dtype) if t.is_floating_point()
             else _values(rnd, g, t.numel(), t.dtype, False)) for k, t in prev.items())) for _ in range(K)]
        for i, (n, d) in enumerate(raw):
            srv.add_local_trained_result(i, d, n)
        out = OrderedDict((k, t.cpu().clone()) for k, t in srv.aggregate().items())
        host = copy.deepcopy(raw)
        if opt == "sgd":
            exp = orc.fedopt_round(prev, names, host, lr, mom, state)
        elif opt in ("adam", "adamw"):
            exp = orc.fedopt_adam_round(prev, names, host, lr, state, r + 1, sqrt="ieee",
                                        weight_decay=0.01 if opt == "adamw" else 0.0)
        elif opt == "adagrad":
            exp = orc.fedopt_adagrad_round(prev, names, host, lr, state, sqrt="ieee")
        elif opt == "rmsprop":
            exp = orc.fedopt_rmsprop_round(prev, names, host, lr, state, sqrt="ieee")
        else:
            exp = orc.fedopt_optrepo_round(opt, prev, names, host, lr, state, r + 1, sqrt="ieee")
        assert list(out) == list(exp), what
        for k in exp:
            gu.assert_same(out[k], exp[k], f"{what} round {r} key {k}")
        st = srv.optimizer_state()
        for k in names:
            if opt == "sgd" and mom:
                gu.assert_same(st["momentum_buffer"][k].cpu().reshape(-1), torch.from_numpy(state[k]).reshape(-1),
                               f"{what} round {r} momentum {k}")
            elif opt in ("adam", "adamw"):
                gu.assert_same(st["exp_avg"][k].cpu().reshape(-1), torch.from_numpy(state[k][0]), f"{what} m {k}")
                gu.assert_same(st["exp_avg_sq"][k].cpu().reshape(-1), torch.from_numpy(state[k][1]), f"{what} v {k}")
            elif opt in ("adagrad", "rmsprop"):
                name = "sum" if opt == "adagrad" else "square_avg"
                gu.assert_same(st[name][k].cpu().reshape(-1), torch.from_numpy(state[k]), f"{what} {name} {k}")
            elif opt in orc.OPTREPO_STATE:
                for name in orc.OPTREPO_STATE[opt]:
                    gu.assert_same(st[name][k].cpu().reshape(-1), torch.from_numpy(state[k][name]),
                                   f"{what} {name} {k}")
        prev = out


class _Holder(torch.nn.Module):
    """A server model whose state dict is exactly the fuzz case's keys."""

    def __init__(self, entries):
        super().__init__()
        for k, s, dt in entries:
            self.register_buffer(k, torch.zeros(s, dtype=dt))


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 60 * _SCALE)))
def test_random_cross_silo_rounds_match_the_oracle(seed, cuda_device):
    """The cross-silo mirror (fedml_aggregator.py:58-106) over three rounds on
    one server: random layout, client count and arrival order; now and then an
    update with an extra key (moved key by key), a non-contiguous tensor, one
    already on the GPU, or a value rebound after arrival (a hook); the server
    model on the host (the buffer-wise D2H) or on the GPU; one to three
    shards (args.fedagg_devices).  Every round's
    average and the model's state after set_model_params match the oracle."""
    from fedml_amd.cross_silo import FedMLAggregator
    from fedml_amd.server_aggregator import MI355XServerAggregator

    rnd = random.Random(4000 + seed)
    g = torch.Generator().manual_seed(4000 + seed)
    opt = rnd.choice(["FedAvg", "FedAvg", "FedProx", "FedAvg_seq"])
    K = rnd.choice([1, 2, 3, 6, 17, 40])
    budget = (12 << 20) // K
    entries = []
    for j in range(rnd.randint(1, 6)):
        n = rnd.choice([x for x in _LENGTHS if x <= budget] or [1])
        budget = max(1, budget - n)
        shape = (n,) if n < 4 or n % 2 else (2, n // 2)
        entries.append((f"k{j}", shape, rnd.choice(_SUMMED)))
    model = _Holder(entries)
    on_gpu = rnd.random() < 0.4
    if on_gpu:
        model = model.to(cuda_device)
    args = _Args(opt, None)
    G = random.Random(seed + 99).choice([1, 1, 2, 3])  # shards of a MultiDeviceBucket, one GPU standing in
    if G > 1:
        args.fedagg_devices = [cuda_device] * G
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, cuda_device, args, MI355XServerAggregator(model, args))
    what = f"cross-silo seed {seed}: G={G} {opt} K={K} model_on_gpu={on_gpu} keys={[(k, s, str(d)) for k, s, d in entries]}"
    for r in range(3):
        raw, quirks = [], []
        for i in range(K):
            d = OrderedDict((k, _values(rnd, g, int(np.prod(s)), dt, False).reshape(s)) for k, s, dt in entries)
            q = rnd.choice(["plain"] * 8 + ["extra", "strided", "device", "hook"])
            if q == "extra" and i > 0:
                d["unused.extra"] = torch.ones(3)
            elif q == "strided":
                k, s, dt = rnd.choice(entries)
                d[k] = torch.stack([d[k], d[k]], -1)[..., 0]  # same values, non-contiguous
            quirks.append(q)
            raw.append((rnd.choice([1, 3, 64, 2.5]), d))
        host = copy.deepcopy(raw)
        for i in rnd.sample(range(K), K):
            n, d = raw[i]
            if quirks[i] == "device":
                d = OrderedDict((k, t.to(cuda_device)) for k, t in d.items())
            server.add_local_trained_result(i, d, n)
            if quirks[i] == "hook":
                k = rnd.choice(entries)[0]
                d[k] = d[k] * 2 if d[k].is_floating_point() else d[k] + 1
                host[i][1][k] = host[i][1][k] * 2 if host[i][1][k].is_floating_point() else host[i][1][k] + 1
        assert server.check_whether_all_receive(), what
        exp = orc.agg(_Args(opt, None), host)
        averaged, _, _ = server.aggregate()
        tag = f"{what} round {r} quirks={quirks}"
        for k in exp:
            gu.assert_same(averaged[k].cpu(), exp[k], f"{tag} key {k}")
        sd = model.state_dict()
        for k, s, dt in entries:
            gu.assert_same(sd[k].cpu(), torch.zeros(s, dtype=dt).copy_(exp[k]), f"{tag} model {k}")


class _DefArgs:
    def __init__(self, defense, **kw):
        self.federated_optimizer = "FedAvg"
        self.enable_defense = True
        self.defense_type = defense
        for k, v in kw.items():
            setattr(self, k, v)


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 60 * _SCALE)))
def test_random_defended_round_matches_the_oracle(seed, cuda_device):
    """The defenses on the hot path's kernels (fedml_defender.py:131-171):
    coordinate-wise median (mixed 16/32-bit weight keys, NaN now and then),
    trimmed mean, Krum / multi-Krum with scaled outliers, norm-diff clipping
    against the server model; random K, sizes, sample counts and residency.
    The defended average matches the oracle bit for bit, errors by type."""
    from fedml_amd.server_aggregator import MI355XServerAggregator

    rnd = random.Random(5000 + seed)
    g = torch.Generator().manual_seed(5000 + seed)
    defense = rnd.choice(["wise_median", "wise_median", "trimmed_mean", "krum", "multikrum", "norm_diff_clipping"])
    K = rnd.choice([1, 2, 3, 5, 9, 16, 33, 64, 129, 300] if defense in ("wise_median", "trimmed_mean")
                   else [4, 6, 9, 16, 20, 33])
    budget = (6 << 20) // K
    entries = []
    for j in range(rnd.randint(1, 4)):
        n = rnd.choice([x for x in _LENGTHS if 0 < x <= budget] or [1])
        budget = max(1, budget - n)
        dt = rnd.choice([torch.float32, torch.bfloat16, torch.float16]) if defense == "wise_median" else torch.float32
        entries.append((f"layer{j}_weight", (n,), dt))
    if defense != "wise_median" and rnd.random() < 0.5:
        entries += [("bn_running_mean", (7,), torch.float32), ("bn_num_batches_tracked", (), torch.int64)]
    special = defense == "wise_median" and rnd.random() < 0.2
    kw = {}
    if defense == "trimmed_mean":
        kw["beta"] = rnd.choice([0.0, 0.1, 0.2, 0.3, 0.49])
    elif defense in ("krum", "multikrum"):
        f = rnd.randint(0, max(0, (K - 4) // 2))
        kw["byzantine_client_num"] = f
        kw["krum_param_m"] = rnd.randint(1, max(1, K - 2 * f - 2)) if defense == "multikrum" else 1
    elif defense == "norm_diff_clipping":
        kw["norm_bound"] = rnd.choice([0.01, 0.5, 5.0, 1e3])
    args = _DefArgs(defense, **kw)
    model = _Holder(entries)
    with torch.no_grad():
        for t in model.state_dict().values():
            t.copy_(_values(rnd, g, t.numel(), t.dtype, False).reshape(t.shape))
    raw = []
    outliers = set(rnd.sample(range(K), rnd.randint(0, K // 4))) if defense in ("krum", "multikrum") else set()
    for i in range(K):
        d = OrderedDict((k, _values(rnd, g, s[0] if s else 1, dt, special).reshape(s)) for k, s, dt in entries)
        if i in outliers:
            d = OrderedDict((k, t * 20 if t.is_floating_point() else t) for k, t in d.items())
        raw.append((rnd.choice([1, 2, 10, 37, 5.5]), d))
    device = rnd.random() < 0.5
    what = f"{defense} seed {seed}: K={K} {kw} device={device} keys={[(k, s, str(d)) for k, s, d in entries]}"
    host = copy.deepcopy(raw)
    gmodel = OrderedDict((k, t.clone()) for k, t in model.state_dict().items())
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    agg = MI355XServerAggregator(model, args)
    try:
        exp = orc.defended_agg(args, host, gmodel)
    except Exception as e:  # noqa: BLE001
        with pytest.raises(type(e)):
            lst, _ = agg.on_before_aggregation(raw)
            agg.on_after_aggregation(agg.aggregate(lst))
        return
    lst, idxs = agg.on_before_aggregation(raw)
    assert idxs == list(range(K)), what
    got = agg.on_after_aggregation(agg.aggregate(lst))
    assert list(got) == list(exp), what
    for k in exp:
        gu.assert_same(got[k].cpu(), exp[k].reshape(got[k].shape), f"{what} key {k}")


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 40 * _SCALE)))
def test_random_multidevice_round_matches_the_oracle(seed, cuda_device):
    """The same random rounds with args.fedagg_devices listing 2-4 shards (one
    GPU standing in for several, as tests/test_gpu_multidev.py): whole keys
    per shard, each reduced where it lives (fedml_amd.multidev)."""
    opt, K, keys, raw, acc, device = _case(6000 + seed)
    G = random.Random(seed).choice([2, 3, 4])
    what = f"multidev seed {seed}: G={G} {opt} K={K} acc={acc} device={device} keys={[(k, s, str(d)) for k, s, d in keys]}"
    host = copy.deepcopy(raw)
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    args = _Args(opt, acc)
    args.fedagg_devices = [cuda_device] * G
    got = FedMLAggOperator.agg(args, raw)
    exp = orc.agg(_Args(opt, None), copy.deepcopy(host))
    assert list(got) == list(exp), what
    ws = [n / sum(n for n, _ in host) for n, _ in host]
    for k, s, dt in keys:
        e = exp[k]
        if acc == "fp32" and dt in (torch.bfloat16, torch.float16):
            e = orc.wsum_acc32([d[k] for _, d in host], ws)
        gu.assert_same(got[k].cpu(), e, f"{what} key {k}")


def _odd(rnd: random.Random, t: torch.Tensor) -> torch.Tensor:
    """The same values in an unusual tensor: non-contiguous, at an odd storage
    offset (an unaligned pointer), or an nn.Parameter (a tensor subclass)."""
    kind = rnd.choice(["strided", "offset", "param"])
    if kind == "strided":
        return torch.stack([t, t], -1)[..., 0]
    if kind == "offset":
        big = torch.empty(t.numel() + 3, dtype=t.dtype, device=t.device)
        big[3:].copy_(t.reshape(-1))
        return big[3:].view(t.shape)
    if not t.is_floating_point():
        return t
    return torch.nn.Parameter(t.clone(), requires_grad=False)


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 60 * _SCALE)))
def test_random_round_with_odd_tensors_matches_the_oracle(seed, cuda_device):
    """The random rounds again with a fifth of the client tensors replaced by
    non-contiguous views, unaligned views or nn.Parameters (the native walker
    declines those; the reference takes them as they are)."""
    opt, K, keys, raw, acc, device = _case(7000 + seed)
    rnd = random.Random(seed)
    what = f"odd seed {seed}: {opt} K={K} acc={acc} device={device} keys={[(k, s, str(d)) for k, s, d in keys]}"
    host = copy.deepcopy(raw)
    if device:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    raw = [(n, OrderedDict((k, _odd(rnd, t) if rnd.random() < 0.2 else t) for k, t in d.items())) for n, d in raw]
    got = FedMLAggOperator.agg(_Args(opt, acc), raw)
    exp = orc.agg(_Args(opt, None), copy.deepcopy(host))
    assert list(got) == list(exp), what
    ws = [n / sum(n for n, _ in host) for n, _ in host]
    for k, s, dt in keys:
        e = exp[k]
        if acc == "fp32" and dt in (torch.bfloat16, torch.float16):
            e = orc.wsum_acc32([d[k] for _, d in host], ws)
        gu.assert_same(got[k].detach().cpu(), e, f"{what} key {k}")


@pytest.mark.parametrize("seed", list(range(_SEED0, _SEED0 + 40 * _SCALE)))
def test_random_bucket_rounds_match_the_oracle(seed, cuda_device):
    """ClientBucket itself over three rounds on the same slots: each client
    arrives in random order through put() (host dict), put() of a device
    dict, or put_encoded() of a FAGG message (pageable or pinned), now and
    then through reduce_to_host; the fp32 accumulation mode too.  FedAvg of
    the slots matches the oracle (integer keys promoted into the fp32 rows,
    as the reference's int64 * float gives float32)."""
    from fedml_amd import wire
    from fedml_amd.bucket import ClientBucket

    rnd = random.Random(8000 + seed)
    g = torch.Generator().manual_seed(8000 + seed)
    K = rnd.choice([1, 2, 5, 16, 33, 100])
    budget = (8 << 20) // K
    entries = []
    for j in range(rnd.randint(1, 5)):
        n = rnd.choice([x for x in _LENGTHS if x <= budget] or [1])
        budget = max(1, budget - n)
        shape = (n,) if n < 4 or n % 2 else (n // 2, 2)
        entries.append((f"k{j}", shape, rnd.choice([torch.float32, torch.bfloat16, torch.float16, torch.float64,
                                                    torch.int64])))
    acc = rnd.choice(["reference", "reference", "fp32"])
    bucket = ClientBucket(entries, K, cuda_device, low_precision_acc=acc)
    what = f"bucket seed {seed}: K={K} acc={acc} keys={[(k, s, str(d)) for k, s, d in entries]}"
    for r in range(3):
        raw = [(rnd.choice([1, 9, 250, 3.5]),
                OrderedDict((k, _values(rnd, g, int(np.prod(s)), dt, rnd.random() < 0.1).reshape(s))
                            for k, s, dt in entries)) for _ in range(K)]
        hows = []
        for i in rnd.sample(range(K), K):
            n, d = raw[i]
            how = rnd.choice(["put", "device", "wire", "wire_pinned"])
            hows.append(how)
            if how == "put":
                bucket.put(i, d, n)
            elif how == "device":
                bucket.put(i, OrderedDict((k, t.to(cuda_device)) for k, t in d.items()), n)
            else:
                m = wire.encode(d, n)
                if how == "wire_pinned":
                    t = torch.empty(len(m), dtype=torch.uint8).pin_memory()
                    t.numpy()[:] = np.frombuffer(m, dtype=np.uint8)
                    m = t.numpy()
                bucket.put_encoded(i, m)
                bucket.wait_ingest()  # the receive buffer is reused by the next message
        to_host = rnd.random() < 0.3
        res = bucket.reduce_to_host(bucket.weights([n for n, _ in raw])) if to_host else bucket.aggregate()
        exp = orc.agg(_Args("FedAvg", None), copy.deepcopy(raw))
        ws = [n / sum(n for n, _ in raw) for n, _ in raw]
        tag = f"{what} round {r} to_host={to_host}"
        assert list(res) == list(exp), tag
        for k, s, dt in entries:
            e = exp[k]
            if acc == "fp32" and dt in (torch.bfloat16, torch.float16):
                e = orc.wsum_acc32([d[k] for _, d in raw], ws)
            gu.assert_same(res[k].cpu(), e, f"{tag} key {k}")
