"""GPU parity of the fused FedOpt server step against the reference's
FedOptAggregator golden vectors (3 rounds, momentum carried across rounds)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import kernels as kn
from fedml_amd.fedopt import FedOptServer
from fedml_amd.synth import fingerprint, host_clients
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("spec", cases.FEDOPT_CASES, ids=lambda s: s["name"])
def test_fedopt_matches_reference(spec, cuda_device):
    meta, arrays = gu.load(spec["name"])
    init = cases.fedopt_global_init(spec)
    gsd = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                      for k, t in init.items())
    server = FedOptServer(gsd, cases.FEDOPT_PARAMS, spec["K"], "sgd", spec["lr"], spec["momentum"], cuda_device)
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        assert server.check_whether_all_receive()
        out = server.aggregate()
        gsd = OrderedDict((k, t.cpu().clone()) for k, t in out.items())
        for k, t in gsd.items():
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            gu.assert_same(t, e, f"{spec['name']} round {r} {k}")


def test_fused_equals_two_kernel_sequence(cuda_device):
    """fedagg_wsum_fedopt_sgd_f32 == fedagg_wsum_f32 then fedagg_fedopt_sgd_f32,
    bit for bit, over 3 rounds at LoRA size (config 5 layout, 64 clients), and
    both == the C oracle on the head and the ragged tail every round (the
    full 64 x 4,194,304 config-5 check is tests/test_gpu_configs.py)."""
    K, N = 64, 1_048_579  # ragged tail on purpose
    g = torch.Generator(device=cuda_device).manual_seed(3)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device) * 0.02
    p0 = torch.randn(N, generator=g, device=cuda_device) * 0.02
    ws = [1.0 / K + (i % 7) * 1e-4 for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_w = kn.upload_f32(ws, cuda_device)
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    pa, ma = p0.clone(), torch.zeros(N, device=cuda_device)
    pb, mb = p0.clone(), torch.zeros(N, device=cuda_device)
    avg = torch.empty(N, device=cuda_device)
    cols = torch.cat([torch.arange(4099), torch.arange(N - 4099, N)]).to(cuda_device)  # head and ragged tail
    hp, hb = p0[cols].cpu().numpy(), None
    for r in range(3):
        kn.wsum_fedopt_sgd(d_ptrs, d_w, K, N, pa, ma, 1.0, 0.9, r == 0, True)
        kn.wsum_ptrs(torch.float32, d_ptrs, d_w, K, N, avg, True)
        kn.fedopt_sgd(pb, mb, avg, 1.0, 0.9, r == 0)
        # the C oracle on those columns: wsum chain, then the fmaf SGD step
        host = rows[:, cols].cpu().numpy()
        hp, hb = orc.fedopt_sgd(hp, orc.c_wsum([host[i] for i in range(K)], ws), hb, 1.0, 0.9, r == 0)
        gu.assert_same(pa[cols].cpu(), torch.from_numpy(hp), f"round {r} param vs oracle")
        gu.assert_same(ma[cols].cpu(), torch.from_numpy(hb), f"round {r} momentum vs oracle")
        rows.mul_(1.01)
    gu.assert_same(pa.cpu(), pb.cpu(), "param")
    gu.assert_same(ma.cpu(), mb.cpu(), "momentum")


def test_fedopt_lora_layout_is_one_launch(cuda_device):
    from fedml_amd.shapes import llama2_7b_lora

    ents = llama2_7b_lora(layers=2)
    sd = OrderedDict((k, torch.zeros(s)) for k, s, _ in ents)
    server = FedOptServer(sd, list(sd.keys()), 4, "sgd", 1.0, 0.9, cuda_device)
    assert len(server.runs) == 1 and server.runs[0][0]


def _golden_state(arrays, r, names):
    """Torch's Adam state after round r (r = -1: before the first step)."""
    if r < 0:
        return {"step": 0}
    st = {"step": r + 1, "exp_avg": OrderedDict(), "exp_avg_sq": OrderedDict()}
    for k in names:
        st["exp_avg"][k] = torch.from_numpy(arrays[f"r{r}:exp_avg:{k}"].copy())
        st["exp_avg_sq"][k] = torch.from_numpy(arrays[f"r{r}:exp_avg_sq:{k}"].copy())
    return st


def _bits(t: torch.Tensor):
    return t.detach().cpu().contiguous().reshape(-1).view(torch.int32)


@pytest.mark.parametrize("spec", cases.FEDOPT_ADAM_CASES, ids=lambda s: s["name"])
def test_fedopt_adam_matches_reference(spec, cuda_device):
    """Each round of FedOptAPI's server Adam, started from the reference's own
    state of the previous round (parameters and optimizer moments):
      - exp_avg / exp_avg_sq and every buffer: bit-identical to torch;
      - parameters: bit-identical to the oracle with a correctly rounded sqrt,
        and within 1 ulp(p) + 2^-21 |step| of torch, whose CPU sqrt (MKL VML)
        is not correctly rounded — the only source of difference."""
    meta, arrays = gu.load(spec["name"])
    names = cases.FEDOPT_PARAMS
    init = cases.fedopt_global_init(spec)
    prev = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                       for k, t in init.items())
    exact = total = 0
    for r in range(spec["rounds"]):
        server = FedOptServer(prev, names, spec["K"], "adam", spec["lr"], 0.0, cuda_device)
        server.load_optimizer_state(_golden_state(arrays, r - 1, names))
        raw = cases.fedopt_round_inputs(spec, prev, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        out = OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items())
        st = server.optimizer_state()
        assert st["step"] == r + 1
        gold = _golden_state(arrays, r, names)
        for k in names:
            gu.assert_same(st["exp_avg"][k].cpu(), gold["exp_avg"][k].reshape(st["exp_avg"][k].shape), f"r{r} m {k}")
            gu.assert_same(st["exp_avg_sq"][k].cpu(), gold["exp_avg_sq"][k].reshape(st["exp_avg_sq"][k].shape),
                           f"r{r} v {k}")
        # oracle, same inputs, IEEE sqrt: bit-exact
        ostate = {k: (_golden_state(arrays, r - 1, names)["exp_avg"][k].numpy(),
                      _golden_state(arrays, r - 1, names)["exp_avg_sq"][k].numpy()) for k in names} if r else {}
        exp = orc.fedopt_adam_round(prev, names, raw, spec["lr"], ostate, r + 1, sqrt="ieee")
        for k, t in out.items():
            gu.assert_same(t, exp[k], f"r{r} oracle {k}")
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            if k in names:
                step = (e.double() - prev[k].double()).abs()
                tol = torch.from_numpy(np.spacing(np.abs(e.numpy()))).double() + step * 2.0 ** -21
                assert ((t.double() - e.double()).abs() <= tol).all(), f"r{r} {k}"
                exact += int((_bits(t) == _bits(e)).sum())
                total += t.numel()
            else:
                gu.assert_same(t, e, f"r{r} {k}")
        prev = OrderedDict((k, gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                           for k, t in init.items())
    assert exact >= 0.98 * total, (exact, total)


def test_fused_adam_vs_oracle_large(cuda_device):
    """Fused Adam at LoRA scale with a ragged tail, 3 rounds, every element
    bit-exact against the C oracle (IEEE sqrt): moments and parameters."""
    K, N = 16, 262_147
    g = torch.Generator(device=cuda_device).manual_seed(9)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device) * 0.02
    p = torch.randn(N, generator=g, device=cuda_device) * 0.02
    m = torch.zeros(N, device=cuda_device)
    v = torch.zeros(N, device=cuda_device)
    ws = [(i + 1.0) for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_w = kn.upload_f32(ws, cuda_device)
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    hp, hm, hv = p.cpu().numpy(), None, None
    for r in range(3):
        avg = orc.wsum([rows[i, :N].cpu() for i in range(K)], ws).numpy()
        kn.wsum_fedopt_adam(d_ptrs, kn.weights_for(ws, torch.float32, cuda_device), K, N, p, m, v,
                            kn.adam_scalars(0.01, 0.9, 0.999, 1e-8, r + 1), r == 0, True)
        hp, hm, hv = orc.fedopt_adam(hp, avg, hm, hv, 0.01, r + 1, sqrt="ieee")
        gu.assert_same(m.cpu(), torch.from_numpy(hm), f"r{r} exp_avg")
        gu.assert_same(v.cpu(), torch.from_numpy(hv), f"r{r} exp_avg_sq")
        gu.assert_same(p.cpu(), torch.from_numpy(hp), f"r{r} param")
        rows.mul_(1.01)
    assert d_w.numel() == K


@pytest.mark.parametrize("spec", cases.FEDOPT_ADAGRAD_CASES, ids=lambda s: s["name"])
def test_fedopt_adagrad_matches_reference(spec, cuda_device):
    """Each round of FedOptAPI's server Adagrad, started from the reference's
    own state of the previous round: state_sum and every buffer bit-identical
    to torch; parameters bit-identical to the oracle with a correctly rounded
    sqrt and within 1 ulp(p) + 2^-21 |step| of torch (CPU sqrt)."""
    meta, arrays = gu.load(spec["name"])
    names = cases.FEDOPT_PARAMS
    init = cases.fedopt_global_init(spec)
    prev = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                       for k, t in init.items())
    exact = total = 0
    for r in range(spec["rounds"]):
        server = FedOptServer(prev, names, spec["K"], "adagrad", spec["lr"], 0.0, cuda_device)
        state = {"step": r}
        if r:
            state["sum"] = OrderedDict((k, torch.from_numpy(arrays[f"r{r - 1}:sum:{k}"].copy())) for k in names)
        server.load_optimizer_state(state)
        raw = cases.fedopt_round_inputs(spec, prev, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        out = OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items())
        st = server.optimizer_state()
        assert st["step"] == r + 1
        for k in names:
            gold = torch.from_numpy(arrays[f"r{r}:sum:{k}"].copy()).reshape(st["sum"][k].shape)
            gu.assert_same(st["sum"][k].cpu(), gold, f"r{r} sum {k}")
        osum = {k: arrays[f"r{r - 1}:sum:{k}"].reshape(-1).copy() for k in names} if r else {}
        exp = orc.fedopt_adagrad_round(prev, names, raw, spec["lr"], osum, sqrt="ieee")
        for k, t in out.items():
            gu.assert_same(t, exp[k], f"r{r} oracle {k}")
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            if k in names:
                step = (e.double() - prev[k].double()).abs()
                tol = torch.from_numpy(np.spacing(np.abs(e.numpy()))).double() + step * 2.0 ** -21
                assert ((t.double() - e.double()).abs() <= tol).all(), f"r{r} {k}"
                exact += int((_bits(t) == _bits(e)).sum())
                total += t.numel()
            else:
                gu.assert_same(t, e, f"r{r} {k}")
        prev = OrderedDict((k, gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                           for k, t in init.items())
    assert exact >= 0.98 * total, (exact, total)


@pytest.mark.parametrize("N", [262_147, 5_000_011])
def test_fused_adagrad_vs_oracle_large(N, cuda_device):
    """Fused Adagrad with a ragged tail (small-tile and mid-tile launches),
    3 rounds, every element bit-exact against the C oracle (IEEE sqrt)."""
    K = 12
    g = torch.Generator(device=cuda_device).manual_seed(N % 101)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device) * 0.02
    p = torch.randn(N, generator=g, device=cuda_device) * 0.02
    acc = torch.zeros(N, device=cuda_device)
    ws = [(i + 2.0) for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    hp, hs = p.cpu().numpy(), None
    for r in range(3):
        avg = orc.wsum([rows[i, :N].cpu() for i in range(K)], ws).numpy()
        kn.wsum_fedopt_adagrad(d_ptrs, kn.weights_for(ws, torch.float32, cuda_device), K, N, p, acc, 0.1, 1e-10, True)
        hp, hs = orc.fedopt_adagrad(hp, avg, hs, 0.1, sqrt="ieee")
        gu.assert_same(acc.cpu(), torch.from_numpy(hs), f"r{r} sum")
        gu.assert_same(p.cpu(), torch.from_numpy(hp), f"r{r} param")
        rows.mul_(1.01)


def test_optimizer_state_round_trip(cuda_device):
    spec = cases.FEDOPT_ADAM_CASES[0]
    init = cases.fedopt_global_init(spec)
    a = FedOptServer(init, cases.FEDOPT_PARAMS, spec["K"], "adam", spec["lr"], 0.0, cuda_device)
    gsd = init
    for r in range(2):
        for i, (n, d) in enumerate(cases.fedopt_round_inputs(spec, gsd, r)):
            a.add_local_trained_result(i, d, n)
        gsd = OrderedDict((k, t.cpu().clone()) for k, t in a.aggregate().items())
    b = FedOptServer(gsd, cases.FEDOPT_PARAMS, spec["K"], "adam", spec["lr"], 0.0, cuda_device)
    b.load_optimizer_state(a.optimizer_state())
    raw = cases.fedopt_round_inputs(spec, gsd, 2)
    for s in (a, b):
        for i, (n, d) in enumerate(raw):
            s.add_local_trained_result(i, d, n)
    oa, ob = a.aggregate(), b.aggregate()
    for k in oa:
        gu.assert_same(oa[k].cpu(), ob[k].cpu(), k)


@pytest.mark.parametrize("opt", ["sgd", "adam", "adagrad"])
def test_sharded_fedopt_single_rank_matches_fused_server(opt, cuda_device):
    """The multi-GPU FedOpt path (client-axis average, then the step on the
    rank's shard through the fused kernel with one source at weight 1.0), run
    on one rank, is bit-identical to the single-GPU fused server over three
    rounds: the same chain, the same step arithmetic."""
    from fedml_amd.sharded import ShardedFedOpt

    entries = [("q.lora_A", (8, 300), torch.float32), ("q.lora_B", (300, 8), torch.float32),
               ("v.lora_A", (8, 77), torch.float32)]
    K = 6
    init = host_clients(entries, 1, seed=5)[0][1]
    srv = FedOptServer(init, [k for k, _, _ in entries], K, opt, 0.5, 0.9, cuda_device)
    flat0 = srv.global_flat[torch.float32].clone()
    L = srv.bucket.groups[torch.float32].length
    sh = None
    for r in range(3):
        raw = host_clients(entries, K, seed=20 + r, round_idx=r)
        for i, (n, d) in enumerate(raw):
            srv.add_local_trained_result(i, d, n)
        srv.aggregate()
        if sh is None:
            sh = ShardedFedOpt(srv.bucket.groups[torch.float32].rows, L, flat0, opt, 0.5, 0.9, chunks=3)
        ns = [n for n, _ in raw]
        sh.aggregate([n / sum(ns) for n in ns])
        torch.cuda.synchronize()
        gu.assert_same(sh.gather_params().cpu(), srv.global_flat[torch.float32][:L].cpu(), f"{opt} round {r}")


def _state_for(opt, arrays, r, names):
    """The reference optimizer's state after round r (r = -1: before the first step)."""
    st = {"step": r + 1}
    if r < 0:
        return st
    bufs = ("square_avg",) if opt == "rmsprop" else ("exp_avg", "exp_avg_sq")
    for b in bufs:
        st[b] = OrderedDict((k, torch.from_numpy(arrays[f"r{r}:{b}:{k}"].copy())) for k in names)
    return st


@pytest.mark.parametrize("spec", cases.FEDOPT_RMSPROP_CASES + cases.FEDOPT_ADAMW_CASES, ids=lambda s: s["name"])
def test_fedopt_rmsprop_adamw_match_reference(spec, cuda_device):
    """Each round of FedOptAPI's server RMSprop (the reference's own flow) and
    AdamW (the same flow with torch.optim.AdamW registered), started from the
    fixture's state of the previous round: optimizer state and buffers
    bit-identical to torch; parameters bit-identical to the oracle with an
    IEEE sqrt and within 1 ulp + 2^-21 |step| of torch (CPU sqrt)."""
    opt = spec["optimizer"]
    meta, arrays = gu.load(spec["name"])
    names = cases.FEDOPT_PARAMS
    init = cases.fedopt_global_init(spec)
    prev = OrderedDict((k, gu.to_tensor(arrays[f"init:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                       for k, t in init.items())
    exact = total = 0
    for r in range(spec["rounds"]):
        server = FedOptServer(prev, names, spec["K"], opt, spec["lr"], 0.0, cuda_device)
        server.load_optimizer_state(_state_for(opt, arrays, r - 1, names))
        raw = cases.fedopt_round_inputs(spec, prev, r)
        assert fingerprint(raw) == meta["rounds"][r]["in_sha256"]
        for i, (n, d) in enumerate(raw):
            server.add_local_trained_result(i, d, n)
        out = OrderedDict((k, t.cpu().clone()) for k, t in server.aggregate().items())
        st = server.optimizer_state()
        gold = _state_for(opt, arrays, r, names)
        for b in [x for x in gold if x != "step"]:
            for k in names:
                gu.assert_same(st[b][k].cpu(), gold[b][k].reshape(st[b][k].shape), f"r{r} {b} {k}")
        prev_state = _state_for(opt, arrays, r - 1, names)
        if opt == "rmsprop":
            ostate = {k: prev_state["square_avg"][k].numpy().reshape(-1) for k in names} if r else {}
            exp = orc.fedopt_rmsprop_round(prev, names, raw, spec["lr"], ostate, sqrt="ieee")
        else:
            ostate = {k: (prev_state["exp_avg"][k].numpy().reshape(-1), prev_state["exp_avg_sq"][k].numpy().reshape(-1))
                      for k in names} if r else {}
            exp = orc.fedopt_adam_round(prev, names, raw, spec["lr"], ostate, r + 1, sqrt="ieee", weight_decay=0.01)
        for k, t in out.items():
            gu.assert_same(t, exp[k], f"r{r} oracle {k}")
            e = gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape)
            if k in names:
                step = (e.double() - prev[k].double()).abs()
                tol = torch.from_numpy(np.spacing(np.abs(e.numpy()))).double() + step * 2.0 ** -21
                assert ((t.double() - e.double()).abs() <= tol).all(), f"r{r} {k}"
                exact += int((_bits(t) == _bits(e)).sum())
                total += t.numel()
            else:
                gu.assert_same(t, e, f"r{r} {k}")
        prev = OrderedDict((k, gu.to_tensor(arrays[f"r{r}:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                           for k, t in init.items())
    assert exact >= 0.98 * total, (exact, total)


@pytest.mark.parametrize("opt", ["rmsprop", "adamw"])
@pytest.mark.parametrize("N", [262_147, 5_000_011])
def test_fused_rmsprop_adamw_vs_oracle_large(opt, N, cuda_device):
    """The fused RMSprop / AdamW launches with a ragged tail (small-tile and
    mid-tile configurations), 3 rounds, every element bit-exact against the
    oracle (IEEE sqrt): state and parameters."""
    K = 10
    g = torch.Generator(device=cuda_device).manual_seed(N % 103)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device) * 0.02
    p = torch.randn(N, generator=g, device=cuda_device) * 0.02
    s1, s2 = torch.zeros(N, device=cuda_device), torch.zeros(N, device=cuda_device)
    ws = [(i + 3.0) for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    hp, h1, h2 = p.cpu().numpy(), None, None
    lr = 0.01
    for r in range(3):
        avg = orc.wsum([rows[i, :N].cpu() for i in range(K)], ws).numpy()
        wt = kn.weights_for(ws, torch.float32, cuda_device)
        if opt == "rmsprop":
            kn.wsum_fedopt_rmsprop(d_ptrs, wt, K, N, p, s1, lr, 0.99, 1e-8, True)
            hp, h1 = orc.fedopt_rmsprop(hp, avg, h1, lr, sqrt="ieee")
        else:
            kn.wsum_fedopt_adamw(d_ptrs, wt, K, N, p, s1, s2, kn.adam_scalars(lr, 0.9, 0.999, 1e-8, r + 1),
                                 1 - lr * 0.01, r == 0, True)
            hp, h1, h2 = orc.fedopt_adam(hp, avg, h1, h2, lr, r + 1, sqrt="ieee", weight_decay=0.01)
            gu.assert_same(s2.cpu(), torch.from_numpy(h2), f"r{r} exp_avg_sq")
        gu.assert_same(s1.cpu(), torch.from_numpy(h1), f"r{r} state")
        gu.assert_same(p.cpu(), torch.from_numpy(hp), f"r{r} param")
        rows.mul_(1.01)
