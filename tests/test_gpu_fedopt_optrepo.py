"""GPU parity of the fused server steps of the other elementwise OptRepo
optimizers (sp/fedopt/optrepo.py:10: Adamax, NAdam, RAdam, Adadelta, ASGD,
Rprop) against the reference's FedOptAPI fixtures and the oracle, and of
FedOptServer's aliasing rule against FedOptAggregator's fixtures.

Parity bar:
  - against the oracle with a correctly rounded sqrt: bit-exact, parameters
    and every state buffer;
  - against torch (the fixtures): Adamax, ASGD and Rprop take no sqrt and are
    bit-exact; NAdam / RAdam keep exp_avg / exp_avg_sq bit-exact, Adadelta its
    square_avg; the parameters of those three (and Adadelta's acc_delta, built
    from a square root) differ from torch's MKL sqrt by its rounding only:
    |d| <= 2 ulp(x) + 2^-20 |step| (acc_delta: 2^-20 |acc_delta|)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import fedopt as fo
from fedml_amd import kernels as kn
from fedml_amd.fedopt import FedOptServer
from fedml_amd.synth import fingerprint, host_clients
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu

SCALARS = {"nadam": ("mu_product",), "asgd": ("eta", "mu")}
NO_SQRT = ("adamax", "asgd", "rprop")
EXACT_STATE = {"adamax": ("exp_avg", "exp_inf"), "nadam": ("exp_avg", "exp_avg_sq"),
               "radam": ("exp_avg", "exp_avg_sq"), "adadelta": ("square_avg",), "asgd": ("ax",),
               "rprop": ("prev", "step_size")}


def _state(opt, arrays, r, names):
    """torch's optimizer state after round r (r = -1: before the first step),
    in FedOptServer.load_optimizer_state's form."""
    st = {"step": r + 1}
    if r < 0:
        return st
    for b in fo.OPTREPO_STATE[opt] + SCALARS.get(opt, ()):
        st[b] = OrderedDict((k, torch.from_numpy(arrays[f"r{r}:{b}:{k}"].copy())) for k in names)
    return st


def _oracle_state(opt, st, names, lr):
    """The same state as the oracle's per-parameter dicts."""
    out = {}
    if st["step"] == 0:
        return out
    for k in names:
        d = {b: st[b][k].numpy().reshape(-1).astype(np.float32).copy() for b in fo.OPTREPO_STATE[opt]}
        for b in SCALARS.get(opt, ()):
            d[b] = np.float32(st[b][k].item())
        out[k] = d
    return out


def _bits(t: torch.Tensor):
    return t.detach().cpu().contiguous().reshape(-1).view(torch.int32)


@pytest.mark.parametrize("spec", cases.FEDOPT_OPTREPO_CASES, ids=lambda s: s["name"])
def test_fedopt_optrepo_matches_reference(spec, cuda_device):
    """Each round of FedOptAPI's server step, started from the reference's own
    state of the previous round (parameters, buffers, fp32 scalar states)."""
    opt = spec["optimizer"]
    meta, arrays = gu.load(spec["name"])
    names = cases.FEDOPT_PARAMS
    init = cases.fedopt_global_init(spec)
    prev = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                       for k, t in init.items())
    exact = total = 0
    for r in range(spec["rounds"]):
        server = FedOptServer(prev, names, spec["K"], opt, spec["lr"], 0.0, cuda_device)
        before = _state(opt, arrays, r - 1, names)
        server.load_optimizer_state(before)
        raw = cases.fedopt_round_inputs(spec, prev, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        out = OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items())
        st = server.optimizer_state()
        assert st["step"] == r + 1
        gold = _state(opt, arrays, r, names)
        for k in names:
            for b in EXACT_STATE[opt]:
                gu.assert_same(st[b][k].cpu(), gold[b][k].reshape(st[b][k].shape), f"r{r} {b} {k}")
            if opt == "adadelta":  # acc_delta = fma(c d, d, acc rho), d built from two square roots
                a, e = st["acc_delta"][k].cpu().double(), gold["acc_delta"][k].reshape(st["acc_delta"][k].shape).double()
                assert ((a - e).abs() <= e.abs() * 2.0 ** -20).all(), f"r{r} acc_delta {k}"
        for b in SCALARS.get(opt, ()):
            assert np.float32(st[b]) == np.float32(gold[b][names[0]].item()), (r, b)
        # the oracle from the same state, IEEE sqrt: bit-exact
        ostate = _oracle_state(opt, before, names, spec["lr"])
        exp = orc.fedopt_optrepo_round(opt, prev, names, raw, spec["lr"], ostate, r + 1, sqrt="ieee")
        for k, t in out.items():
            gu.assert_same(t, exp[k], f"r{r} oracle {k}")
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            if k in names and opt not in NO_SQRT:
                step = (e.double() - prev[k].double()).abs()
                tol = 2 * torch.from_numpy(np.spacing(np.abs(e.numpy()))).double() + step * 2.0 ** -20
                assert ((t.double() - e.double()).abs() <= tol).all(), f"r{r} {k}"
                exact += int((_bits(t) == _bits(e)).sum())
                total += t.numel()
            else:
                gu.assert_same(t, e, f"r{r} {k}")
        prev = OrderedDict((k, gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                           for k, t in init.items())
    if total:
        assert exact >= 0.95 * total, (exact, total)


@pytest.mark.parametrize("opt", list(fo.OPTREPO_STATE))
@pytest.mark.parametrize("N", [262_147, 5_000_011])
def test_fused_optrepo_vs_oracle_large(opt, N, cuda_device):
    """The fused launches with a ragged tail (small- and mid-tile
    configurations), specials in one client (NaN, +-inf, denormals, -0),
    steps 1, 2, 6, 7 (RAdam's plain and rectified branches): every element of
    the parameters and the state bit-exact against the oracle (IEEE sqrt)."""
    K, lr = 10, 0.01
    g = torch.Generator(device=cuda_device).manual_seed(N % 107)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device) * 0.02
    rows[3, :6] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e-40, -0.0, 3e38], device=cuda_device)
    p = torch.randn(N, generator=g, device=cuda_device) * 0.02
    names = fo.OPTREPO_STATE[opt]
    dev_state = {b: torch.zeros(N, device=cuda_device) for b in names}
    if opt == "rprop":
        dev_state["step_size"].fill_(lr)
    ost = orc.optrepo_init(opt, N, lr)
    carry = fo.optrepo_carry(opt, lr)
    ws = [(i + 3.0) for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    hp = p.cpu().numpy()
    for step in (1, 2, 6, 7):
        avg = orc.wsum([rows[i, :N].cpu() for i in range(K)], ws).numpy()
        sc = kn.optrepo_scalars(opt, lr, step, carry)
        kn.wsum_fedopt_optrepo(opt, d_ptrs, kn.weights_for(ws, torch.float32, cuda_device), K, N, p,
                               dev_state[names[0]], dev_state[names[-1]] if len(names) > 1 else None, sc, True)
        hp = orc.fedopt_step(opt, hp, avg, ost, lr, step, sqrt="ieee")
        for b in names:
            gu.assert_same(dev_state[b].cpu(), torch.from_numpy(ost[b]), f"step {step} {b}")
        gu.assert_same(p.cpu(), torch.from_numpy(hp), f"step {step} param")
        for i, b in enumerate(SCALARS.get(opt, ())):
            assert np.float32(carry[i]) == np.float32(ost[b]), (step, b)
        rows.mul_(1.01)


@pytest.mark.parametrize("opt", list(fo.OPTREPO_STATE))
def test_sharded_fedopt_single_rank_matches_fused_server(opt, cuda_device):
    """ShardedFedOpt (client-axis average, then the step on the rank's shard
    through the fused kernel with one source at weight 1.0) on one rank is
    bit-identical to FedOptServer over three rounds."""
    from fedml_amd.sharded import ShardedFedOpt

    entries = [("q.lora_A", (8, 300), torch.float32), ("q.lora_B", (300, 8), torch.float32),
               ("v.lora_A", (8, 77), torch.float32)]
    K = 6
    init = host_clients(entries, 1, seed=5)[0][1]
    srv = FedOptServer(init, [k for k, _, _ in entries], K, opt, 0.5, 0.0, cuda_device)
    flat0 = srv.global_flat[torch.float32].clone()
    L = srv.bucket.groups[torch.float32].length
    sh = None
    for r in range(3):
        raw = host_clients(entries, K, seed=20 + r, round_idx=r)
        for i, (n, d) in enumerate(raw):
            srv.add_local_trained_result(i, d, n)
        srv.aggregate()
        if sh is None:
            sh = ShardedFedOpt(srv.bucket.groups[torch.float32].rows, L, flat0, opt, 0.5, 0.0, chunks=3)
        ns = [n for n, _ in raw]
        sh.aggregate([n / sum(ns) for n in ns])
        torch.cuda.synchronize()
        gu.assert_same(sh.gather_params().cpu(), srv.global_flat[torch.float32][:L].cpu(), f"{opt} round {r}")


@pytest.mark.parametrize("opt", ["nadam", "asgd", "rprop"])
def test_optrepo_state_round_trip(opt, cuda_device):
    """optimizer_state() / load_optimizer_state() carry the buffers AND the
    fp32 scalar states: a second server resumed from the first's state
    continues bit-identically."""
    spec = cases.FEDOPT_ADAM_CASES[0]
    init = cases.fedopt_global_init(spec)
    a = FedOptServer(init, cases.FEDOPT_PARAMS, spec["K"], opt, 0.01, 0.0, cuda_device)
    gsd = init
    for r in range(2):
        for i, (n, d) in enumerate(cases.fedopt_round_inputs(spec, gsd, r)):
            a.add_local_trained_result(i, d, n)
        gsd = OrderedDict((k, t.cpu().clone()) for k, t in a.aggregate().items())
    b = FedOptServer(gsd, cases.FEDOPT_PARAMS, spec["K"], opt, 0.01, 0.0, cuda_device)
    b.load_optimizer_state(a.optimizer_state())
    raw = cases.fedopt_round_inputs(spec, gsd, 2)
    for s in (a, b):
        for i, (n, d) in enumerate(raw):
            s.add_local_trained_result(i, d, n)
    oa, ob = a.aggregate(), b.aggregate()
    for k in oa:
        gu.assert_same(oa[k].cpu(), ob[k].cpu(), k)


@pytest.mark.parametrize("spec", cases.FEDOPT_ALIAS_CASES, ids=lambda s: s["name"])
@pytest.mark.parametrize("shards", [1, 2])
def test_fedopt_alias_matches_reference(spec, shards, cuda_device):
    """FedOptAggregator.aggregate with index 0's dict object added again
    (FedOptAggregator.py:93-101 then reads the running average there):
    FedOptServer (and MultiDeviceFedOptServer over two shards of the one GPU)
    bit-identical to the reference's rounds."""
    from fedml_amd.fedopt import MultiDeviceFedOptServer

    meta, arrays = gu.load(spec["name"])
    init = cases.fedopt_global_init(spec)
    gsd = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                      for k, t in init.items())
    if shards == 1:
        server = FedOptServer(gsd, cases.FEDOPT_PARAMS, spec["K"], "sgd", spec["lr"], spec["momentum"], cuda_device)
    else:
        server = MultiDeviceFedOptServer(gsd, cases.FEDOPT_PARAMS, spec["K"], "sgd", spec["lr"], spec["momentum"],
                                         [cuda_device] * shards)
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for j in spec["alias_of_0"]:
            raw[j] = (raw[j][0], raw[0][1])
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        out = server.aggregate()
        gsd = OrderedDict((k, t.cpu().clone()) for k, t in out.items())
        for k, t in gsd.items():
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            gu.assert_same(t, e, f"{spec['name']} round {r} {k}")


def test_fedopt_alias_differs_from_copies(cuda_device):
    """The aliasing rule is not vacuous: the same round with index 0's dict
    COPIED (a distinct object of equal values) gives a different model."""
    spec = cases.FEDOPT_ALIAS_CASES[0]
    init = cases.fedopt_global_init(spec)
    outs = []
    for copy_it in (False, True):
        server = FedOptServer(init, cases.FEDOPT_PARAMS, spec["K"], "sgd", spec["lr"], spec["momentum"], cuda_device)
        raw = cases.fedopt_round_inputs(spec, init, 0)
        for j in spec["alias_of_0"]:
            d0 = raw[0][1]
            raw[j] = (raw[j][0], OrderedDict((k, t.clone()) for k, t in d0.items()) if copy_it else d0)
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        outs.append(OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items()))
    assert any(not torch.equal(outs[0][k], outs[1][k]) for k in cases.FEDOPT_PARAMS)
