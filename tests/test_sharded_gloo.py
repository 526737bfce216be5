"""Multi-rank partitioning, exercised on CPU with gloo (world_size 2 and 3).

The GPU run uses RCCL and the HIP kernels; here the same partitioning code
runs with host rows and the oracle as the per-rank reducer, so chunking,
shard ownership, the reduce-scatter call pattern and reassembly are all
checked without a GPU.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import traceback
from collections import OrderedDict

import numpy as np
import pytest
import torch
import torch.distributed as dist

from fedml_amd.sharded import ClientAxisAggregator, ParamAxisAggregator, shard_range
from oracle import fedavg_oracle as orc


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clients(K: int, L: int) -> torch.Tensor:
    rng = np.random.default_rng(1234)
    base = rng.standard_normal(L, dtype=np.float32) * np.float32(0.05)
    rows = np.stack([base + np.float32(0.01) * rng.standard_normal(L, dtype=np.float32) for _ in range(K)])
    return torch.from_numpy(rows)


def _oracle_reducer(rows, weights, out):
    out.copy_(orc.wsum([rows[i].contiguous() for i in range(rows.shape[0])], weights))


def _worker(rank, world, port, K_local, L, chunks, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        K = K_local * world
        allrows = _clients(K, L)
        ns = [int(v) for v in np.random.default_rng(7).integers(100, 1001, K)]
        tot = sum(ns)
        ws = [n / tot for n in ns]
        # client axis: this rank owns clients [rank*K_local, (rank+1)*K_local)
        mine = allrows[rank * K_local:(rank + 1) * K_local].clone()
        agg = ClientAxisAggregator(mine, L, chunks=chunks, reducer=_oracle_reducer)
        agg.aggregate(ws[rank * K_local:(rank + 1) * K_local])
        full = agg.gather_full()
        # param axis: this rank owns columns [lo, hi) of every client
        lo, hi = shard_range(L, world, rank)
        pagg = ParamAxisAggregator(allrows[:, lo:hi].contiguous(), hi - lo, reducer=_oracle_reducer)
        pshard = pagg.aggregate(ws).clone()
        sizes = [torch.tensor([0]) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([hi - lo]))
        maxn = max(int(s) for s in sizes)
        buf = torch.zeros(maxn)
        buf[:hi - lo] = pshard
        parts = [torch.zeros(maxn) for _ in range(world)]
        dist.all_gather(parts, buf)
        pfull = torch.cat([parts[r][:int(sizes[r])] for r in range(world)])
        q.put((rank, full.numpy().copy(), pfull.numpy().copy(), agg.owned_ranges(), None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, None, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world,K_local,L,chunks", [(2, 4, 10_001, 3), (3, 3, 4_097, 8), (2, 1, 65, 8),
                                                      (4, 2, 3_001, 4), (8, 1, 2_049, 8)])
def test_client_and_param_axis(world, K_local, L, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K_local, L, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, full, pfull, owned, err = q.get(timeout=120)
        assert err is None, err
        results[rank] = (full, pfull, owned)
    for p in procs:
        p.join(timeout=60)
    K = K_local * world
    allrows = _clients(K, L)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 1001, K)]
    ws = [n / sum(ns) for n in ns]
    chain = orc.wsum([allrows[i] for i in range(K)], ws).numpy()
    partials = [orc.wsum([allrows[i] for i in range(r * K_local, (r + 1) * K_local)],
                         ws[r * K_local:(r + 1) * K_local]).numpy() for r in range(world)]
    for r in range(world):
        full, pfull, owned = results[r]
        # parameter axis: bit-exact with the single-GPU chain
        assert np.array_equal(pfull.view(np.uint32), chain.view(np.uint32))
        # client axis: identical on every rank, and within the stated bound
        assert np.array_equal(full.view(np.uint32), results[0][0].view(np.uint32))
        terms = np.zeros(L, dtype=np.float64)
        for i in range(K):
            terms += np.abs(allrows[i].numpy().astype(np.float64) * np.float32(ws[i]))
        bound = ClientAxisAggregator.tolerance(torch.from_numpy(terms), K, world).numpy()
        assert np.all(np.abs(full.astype(np.float64) - chain.astype(np.float64)) <= bound)
        if world == 2:  # two partials: the reduce-scatter sum is one rounding
            assert np.array_equal(full.view(np.uint32), (partials[0] + partials[1]).view(np.uint32))
        # ownership: disjoint pieces that tile the padded axis
        for a, b in owned:
            assert b > a
    covered = sorted(rng for r in range(world) for rng in results[r][2])
    for (a0, b0), (a1, b1) in zip(covered, covered[1:]):
        assert b0 == a1
    assert covered[0][0] == 0 and covered[-1][1] >= L


def test_shard_range_tiles_axis():
    for n in (0, 1, 63, 64, 65, 25_610_152):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
                assert b0 == a1
            for a, _ in spans:
                assert a % 64 == 0 or a == n


def _sgd_stepper(lr, momentum):
    """torch.optim.SGD's update on flat host tensors (grad = p_old - avg)."""
    def step(param, state, avg):
        grad = param - avg
        if momentum:
            buf = state.get("momentum_buffer")
            if buf is None or not state.get("_started"):
                state["momentum_buffer"] = grad.clone()
                state["_started"] = True
            else:
                buf.mul_(momentum).add_(grad)
            grad = state["momentum_buffer"]
        param.add_(grad, alpha=-lr)
    return step


def _fedopt_worker(rank, world, port, K_local, L, chunks, q):
    try:
        from fedml_amd.sharded import ShardedFedOpt

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        K = K_local * world
        g0 = torch.from_numpy(np.random.default_rng(99).standard_normal(L, dtype=np.float32))
        srv = ShardedFedOpt(torch.zeros(K_local, L), L, g0, "sgd", lr=0.7, momentum=0.9, chunks=chunks,
                            reducer=_oracle_reducer, stepper=_sgd_stepper(0.7, 0.9))
        out = []
        for r in range(2):
            allrows = _clients(K, L) + r  # a different round
            srv.agg.rows = allrows[rank * K_local:(rank + 1) * K_local].clone()
            ns = [int(v) for v in np.random.default_rng(7 + r).integers(100, 1001, K)]
            ws = [n / sum(ns) for n in ns]
            srv.aggregate(ws[rank * K_local:(rank + 1) * K_local])
            out.append((srv.agg.gather_full().numpy().copy(), srv.gather_params().numpy().copy()))
        q.put((rank, out, None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world,K_local,L,chunks", [(2, 3, 5_003, 3), (3, 2, 700, 8)])
def test_sharded_fedopt(world, K_local, L, chunks):
    """Config 5's multi-GPU FedOpt: client-axis average, then the server SGD
    (momentum 0.9) step on each rank's shard with sharded state.  The gathered
    parameters equal the same step applied to the full gathered average, over
    two rounds (state carried), on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fedopt_worker, args=(r, world, port, K_local, L, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, out, err in res:
        assert err is None, err
    g0 = torch.from_numpy(np.random.default_rng(99).standard_normal(L, dtype=np.float32))
    p, state = g0.clone(), {}
    step = _sgd_stepper(0.7, 0.9)
    for r in range(2):
        avg = torch.from_numpy(res[0][1][r][0])
        step(p, state, avg)
        for rank, out, _ in res:
            np.testing.assert_array_equal(out[r][0], res[0][1][r][0])  # every rank gathers the same average
            np.testing.assert_array_equal(out[r][1], p.numpy())


def _bn_rounds(spec_name):
    """The reference's own FedOpt rounds on its BatchNorm model (fixture
    fedopt_sgd_m09_*): per round, the clients' flat fp32 rows (integer
    counters promoted, as the bucket stores them) built from the fixture's
    global model of the previous round, and the fixture's result."""
    import cases
    import golden_util as gu

    from fedml_amd.layout import RowLayout

    spec = next(c for c in cases.FEDOPT_CASES if c["name"] == spec_name)
    meta, arrays = gu.load(spec_name)
    init = cases.fedopt_global_init(spec)
    lay = RowLayout(cases._entries(cases.FEDOPT_MODEL))
    g = lay.groups[torch.float32]

    def flat(sd):
        out = torch.zeros(g.length, dtype=torch.float32)
        for k, o, n in zip(g.keys, g.offsets, g.numels):
            out[o:o + n] = sd[k].reshape(-1).to(torch.float32)
        return out

    def fixture(tag):
        return OrderedDict((k, gu.to_tensor(arrays[f"{tag}:{k}"], str(t.dtype).replace("torch.", ""), t.shape))
                           for k, t in init.items())

    gsd = fixture("init")
    rounds = []
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        rows = torch.stack([flat(d) for _, d in raw])
        ns = [n for n, _ in raw]
        exp = fixture(f"r{r}")
        rounds.append((rows, ns, exp))
        gsd = exp
    return spec, lay, flat(fixture("init")), rounds


def _bn_worker(rank, world, port, spec_name, chunks, q):
    try:
        from fedml_amd.sharded import ShardedFedOpt, buffer_ranges

        import cases

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        spec, lay, g0, rounds = _bn_rounds(spec_name)
        K = spec["K"]
        per = (K + world - 1) // world
        mine = list(range(rank * per, min(K, (rank + 1) * per)))
        L = lay.groups[torch.float32].length
        srv = ShardedFedOpt(torch.zeros(len(mine), L), L, g0, "sgd", lr=spec["lr"], momentum=spec["momentum"],
                            chunks=chunks, reducer=_oracle_reducer,
                            stepper=_sgd_stepper(spec["lr"], spec["momentum"]),
                            buffers=buffer_ranges(lay, cases.FEDOPT_PARAMS))
        out = []
        for rows, ns, _ in rounds:
            srv.agg.rows = rows[mine].clone()
            ws = [n / sum(ns) for n in ns]
            srv.aggregate([ws[i] for i in mine])
            out.append((srv.agg.gather_full().numpy().copy(), srv.gather_params().numpy().copy()))
        q.put((rank, out, None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("spec_name", ["fedopt_sgd_m09_lr1", "fedopt_sgd_m09_lr1e-3"])
def test_sharded_fedopt_steps_parameters_only(world, spec_name):
    """Multi-GPU FedOpt on the reference's BatchNorm model: only named
    parameters take the SGD(momentum 0.9) step; running stats and the
    promoted num_batches_tracked take the plain average
    (FedOptAggregator.py:118-130).  On one rank the chain order is the
    reference's, so every round equals the reference's fixture bit for bit;
    on 2 and 3 ranks the average's addition order changes, so buffers equal
    the gathered average exactly and parameters stay within a few fp32 ulps
    of the fixture across the three rounds (state carried)."""
    import cases
    import golden_util as gu

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_worker, args=(r, world, port, spec_name, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [err for _, _, err in res if err]
    assert not errs, "\n".join(errs)
    spec, lay, _, rounds = _bn_rounds(spec_name)
    g = lay.groups[torch.float32]
    params = set(cases.FEDOPT_PARAMS)
    for r, (_, _, exp) in enumerate(rounds):
        avg, got = res[0][1][r]
        for rank, out, _ in res:
            np.testing.assert_array_equal(out[r][1], got)  # every rank gathers the same model
        for k, o, n in zip(g.keys, g.offsets, g.numels):
            e = exp[k]
            v = torch.from_numpy(got[o:o + n].copy()).reshape(e.shape)
            if k not in params:  # a buffer: exactly the average, never stepped
                np.testing.assert_array_equal(got[o:o + n], avg[o:o + n])
            if e.dtype == torch.int64:
                v = v.to(torch.int64)  # load_state_dict's truncating copy_
            if world == 1:
                gu.assert_same(v, e, f"{spec_name} round {r} {k}")
            elif e.dtype == torch.int64:
                assert torch.equal(v, e), k
            else:
                tol = 64 * 2.0 ** -24 * (e.abs() + 1e-3)
                assert torch.all((v - e).abs() <= tol), (k, r, (v - e).abs().max())


def _bf16_partial_reducer(rows, weights, out):
    """fedagg_wsum_bf16_f32out restated: bf16 rows widened exactly, the fp32
    chain fl32(acc + fl32(x_i * fl32(w_i))) in client order, NO final
    rounding (the fp32 partial a rank sends into the reduce-scatter)."""
    w32 = [np.float32(w) for w in weights]
    x = [orc.bf16_bits_to_f32(rows[i].contiguous().view(torch.int16).numpy().view(np.uint16))
         for i in range(rows.shape[0])]
    acc = x[0] * w32[0]
    for xi, wi in zip(x[1:], w32[1:]):
        acc = acc + xi * wi
    out.copy_(torch.from_numpy(np.asarray(acc, dtype=np.float32)))


def _bf16_worker(rank, world, port, K_local, L, chunks, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        K = K_local * world
        allrows = _clients(K, L).to(torch.bfloat16)
        ns = [int(v) for v in np.random.default_rng(11).integers(100, 1001, K)]
        ws = [n / sum(ns) for n in ns]
        mine = allrows[rank * K_local:(rank + 1) * K_local].clone()
        agg = ClientAxisAggregator(mine, L, chunks=chunks, reducer=_bf16_partial_reducer)
        agg.aggregate(ws[rank * K_local:(rank + 1) * K_local])
        full32 = agg.gather_full()
        full16 = agg.gather_full(agg.shard_in_model_dtype())
        assert full16.dtype == torch.bfloat16
        q.put((rank, full32.numpy().copy(), full16.view(torch.int16).numpy().copy(), None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world,K_local,L,chunks", [(2, 3, 4_099, 3), (4, 2, 1_031, 8), (4, 128, 4_099, 3)])
def test_client_axis_bf16_rows(world, K_local, L, chunks):
    """Config 4's multi-GPU path at world 2 and 4 (the last case is config
    4's 512 clients over 4 ranks): bf16 rows -> per-rank fp32 partial
    (fedagg_wsum_bf16_f32out) -> fp32 reduce-scatter -> ONE bf16 rounding per
    element (shard_in_model_dtype).  Stated tolerances:

    * vs the one-GPU fp32-accumulate result (fedagg_low_precision_acc="fp32",
      orc.wsum_acc32): the fp32 sums differ by at most the reordering bound
      T = 2(K + ceil(log2 G) + 1)·2^-24·Σ|fl(w_i p_i)|, and each side's
      rounding to bf16 by half a bf16 ulp: |Δ| <= T + 2^-7·|acc32|;
    * vs the exact sum (fp64): |Δ| <= T + 2^-8·|exact| + 2^-24·K·Σ|w_i p_i|;
    * vs the reference's own bf16 chain (a bf16 rounding after every mul and
      add, agg_operator.py:40-44): each bf16 rounding errs by at most
      u = 2^-8 relative, so the chain is within 2^-8·(Σ_k |S_k| +
      Σ_i |w_i p_i|) of the exact sum (S_k its running sums), and |Δ| <= that
      + the exact-sum bound above."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_worker, args=(r, world, port, K_local, L, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, "\n".join(errs)
    K = K_local * world
    allrows = _clients(K, L).to(torch.bfloat16)
    ns = [int(v) for v in np.random.default_rng(11).integers(100, 1001, K)]
    ws = [n / sum(ns) for n in ns]
    x64 = np.stack([orc.bf16_bits_to_f32(allrows[i].view(torch.int16).numpy().view(np.uint16))
                    for i in range(K)]).astype(np.float64)
    w32 = np.array([np.float32(w) for w in ws], dtype=np.float64)
    exact = (x64 * w32[:, None]).sum(0)
    terms = np.abs(x64 * w32[:, None]).sum(0)
    T = ClientAxisAggregator.tolerance(torch.from_numpy(terms), K, world).numpy()
    acc32 = orc.bf16_bits_to_f32(orc.wsum_acc32([allrows[i] for i in range(K)], ws).view(torch.int16)
                                 .numpy().view(np.uint16)).astype(np.float64)
    ref = orc.bf16_bits_to_f32(orc.wsum([allrows[i] for i in range(K)], ws).view(torch.int16)
                               .numpy().view(np.uint16)).astype(np.float64)
    # the reference chain's running sums, for its own error bound
    run = np.zeros(L)
    s_abs = np.zeros(L)
    for i in range(K):
        run = run + x64[i] * w32[i]
        s_abs += np.abs(run)
    for rank, full32, full16, _ in res:
        np.testing.assert_array_equal(full16, res[0][2])  # every rank gathers the same model
        np.testing.assert_array_equal(full32.view(np.uint32), res[0][1].view(np.uint32))
        # the bf16 shard is the RNE rounding of the fp32 shard
        np.testing.assert_array_equal(full16.view(np.uint16), orc.f32_to_bf16_bits(full32))
    got = orc.bf16_bits_to_f32(res[0][2].view(np.uint16)).astype(np.float64)
    assert np.all(np.abs(got - acc32) <= T + 2.0 ** -7 * np.abs(acc32))
    b_exact = T + 2.0 ** -8 * np.abs(exact) + 2.0 ** -24 * K * terms
    assert np.all(np.abs(got - exact) <= b_exact)
    assert np.all(np.abs(got - ref) <= b_exact + 2.0 ** -8 * (s_abs + terms))
    if world == 2:  # two partials: the reduce-scatter sum is one fp32 rounding, then one bf16 rounding
        parts = []
        for r in range(world):
            out = torch.empty(L)
            _bf16_partial_reducer(allrows[r * K_local:(r + 1) * K_local], ws[r * K_local:(r + 1) * K_local], out)
            parts.append(out.numpy())
        np.testing.assert_array_equal(res[0][1].view(np.uint32), (parts[0] + parts[1]).view(np.uint32))
