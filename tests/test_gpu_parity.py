"""GPU parity: the HIP path against the reference's golden vectors and the oracle.

Every test here calls libfedagg.so through the C ABI (via fedml_amd) on an
MI355X and compares bit for bit (NaN == NaN) unless it states a tolerance.
"""
from __future__ import annotations

import copy
from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import agg_operator as ao
from fedml_amd import kernels as kn
from fedml_amd import shapes
from fedml_amd.bucket import ClientBucket
from fedml_amd.synth import host_clients
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu

AGG_CASES = [c["name"] for c in cases.CASES]


def _to_device(raw, dev):
    out = []
    for item in raw:
        out.append((item[0],) + tuple(OrderedDict((k, t.to(dev)) for k, t in d.items()) for d in item[1:]))
    return out


def _to_device_aliased(raw, dev):
    """_to_device keeping the round's aliasing: a dict (or tensor) object that
    appears several times on the host appears as ONE device object."""
    memo = {}

    def dmove(d):
        if id(d) not in memo:
            memo[id(d)] = OrderedDict((k, tmove(t)) for k, t in d.items())
        return memo[id(d)]

    def tmove(t):
        if id(t) not in memo:
            memo[id(t)] = t.to(dev)
        return memo[id(t)]

    return [(item[0],) + tuple(dmove(d) for d in item[1:]) for item in raw]


def _cpu(res):
    if isinstance(res, tuple):
        return tuple(_cpu(r) for r in res)
    return OrderedDict((k, t.cpu()) for k, t in res.items())


@pytest.mark.parametrize("name", AGG_CASES)
def test_host_inputs_match_reference(name, cuda_device):
    """Reference call shape: CPU state dicts in, CPU state dict out."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    client0, objs = raw[0][1], dict(raw[0][1])
    before = {k: t.clone() for k, t in objs.items()}
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            ao.FedMLAggOperator.agg(cases.Args(spec), raw)
        assert type(ei.value).__name__ == meta["error"]
        return
    third = gu.snapshot_third(raw)
    res = ao.FedMLAggOperator.agg(cases.Args(spec), raw)
    gu.assert_groups(res, meta, arrays, name)
    gu.assert_third_mutation(third, meta, arrays, name)
    first = res[0] if isinstance(res, tuple) else res
    assert (first is client0) == meta["result_is_client0_dict"]
    for o in meta["outputs"]:
        if o["group"] == 0 and o["key"] in objs:
            assert (first[o["key"]] is objs[o["key"]]) == o["is_client0_tensor"], o["key"]
            assert first[o["key"]].device.type == "cpu"
    for k, t in objs.items():  # which of client 0's tensors were mutated in place
        if t.is_floating_point() and torch.isnan(t).any():
            continue
        changed = not torch.equal(t, before[k])
        assert changed == (k in meta["client0_tensors_mutated"]), k


@pytest.mark.parametrize("name", AGG_CASES)
def test_device_inputs_match_reference(name, cuda_device):
    """Server using_gpu: tensors already in HBM, read in place (multi-tensor launch)."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = _to_device(cases.build_inputs(spec), cuda_device)
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            ao.FedMLAggOperator.agg(cases.Args(spec), raw)
        assert type(ei.value).__name__ == meta["error"]
        return
    third = gu.snapshot_third(raw)
    res = ao.FedMLAggOperator.agg(cases.Args(spec), raw)
    first = res[0] if isinstance(res, tuple) else res
    for t in first.values():
        assert t.is_cuda
    gu.assert_groups(_cpu(res), meta, arrays, name)
    gu.assert_third_mutation(third, meta, arrays, name)


ALIAS_CASES = [c["name"] for c in cases.ALIAS_CASES]


@pytest.mark.parametrize("name", ALIAS_CASES)
@pytest.mark.parametrize("where", ["host", "device"])
def test_alias_rounds_match_reference(name, where, cuda_device):
    """A dict (or, for FedAvg_seq, a tensor) of client 0 listed again reads the
    running accumulator in the reference (agg_operator.py:36-44,55-63,121-133);
    the GPU path reproduces it bit for bit, outputs and in-place side effects."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    if where == "device":
        raw = _to_device_aliased(raw, cuda_device)
    client0, objs = raw[0][1], dict(raw[0][1])
    before = {k: t.clone() for k, t in objs.items()}
    third = gu.snapshot_third(raw)
    res = ao.FedMLAggOperator.agg(cases.Args(spec), raw)
    gu.assert_groups(_cpu(res), meta, arrays, name)
    gu.assert_third_mutation(third, meta, arrays, name)
    first = res[0] if isinstance(res, tuple) else res
    assert (first is client0) == meta["result_is_client0_dict"]
    for t in first.values():
        assert t.device.type == ("cuda" if where == "device" else "cpu")
    for k, t in objs.items():
        if t.is_floating_point() and torch.isnan(t).any():
            continue
        assert (not torch.equal(t, before[k])) == (k in meta["client0_tensors_mutated"]), k


def test_alias_known_answer(cuda_device):
    """[(1, d), (1, d), (2, e)], d = [1, 2], e = [3, 4]: [1.8125, 2.625] as the
    reference computes it here (not the naive mean [2.0, 3.0])."""
    class A:
        federated_optimizer = "FedAvg"

    for dev in ("cpu", cuda_device):
        d = OrderedDict(x=torch.tensor([1.0, 2.0], device=dev))
        e = OrderedDict(x=torch.tensor([3.0, 4.0], device=dev))
        res = ao.FedMLAggOperator.agg(A(), [(1, d), (1, d), (2, e)])
        assert res is d and res["x"].cpu().tolist() == [1.8125, 2.625]


def test_alias_partial_overlap_is_refused(cuda_device):
    class A:
        federated_optimizer = "FedAvg_seq"

    buf = torch.arange(8, dtype=torch.float32, device=cuda_device)
    raw = [(1, OrderedDict(x=buf[0:4])), (1, OrderedDict(x=buf[2:6]))]
    with pytest.raises(NotImplementedError):
        ao.FedMLAggOperator.agg(A(), raw)


@pytest.mark.parametrize("name", [c["name"] for c in cases.CASES
                                  if c["optimizer"] == "FedAvg" and not c.get("expect_error")])
def test_bucket_matches_reference(name, cuda_device):
    """The ingest layout: put() each client into its HBM row, one launch per dtype."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    ns = [n for n, _ in raw]
    bucket = ClientBucket(raw[0][1], len(raw), cuda_device)
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    res = bucket.aggregate()
    exp = gu.expected_groups(meta, arrays)[0]
    for k, e in exp.items():
        gu.assert_same(res[k].cpu(), e, f"{name}[{k}]")
    assert bucket.weights(ns) == [n / sum(ns) for n in ns]


def test_resnet50_multi_tensor_vs_oracle(cuda_device):
    """All 320 ResNet-50 keys as separate device tensors: 267 fp32 keys in one
    multi-tensor launch + 53 int64 keys; every element checked against the oracle."""
    entries = shapes.resnet50()
    raw = host_clients(entries, 6, seed=5, round_idx=3)
    exp = orc.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), copy.deepcopy(raw))
    res = ao.FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), _to_device(raw, cuda_device))
    assert list(res.keys()) == [e[0] for e in entries]
    for k in exp:
        gu.assert_same(res[k].cpu(), exp[k], k)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_resnet50_low_precision_multi_tensor_vs_oracle(dtype, cuda_device):
    """ResNet-50 key shapes held in bf16/f16 as separate device tensors: one
    multi-tensor launch for the float keys (bf16/f16 reference chain), one for
    the 53 int64 keys (fp32 outputs); bit-exact against the oracle."""
    entries = [(k, s, dtype if dt == torch.float32 else dt) for k, s, dt in shapes.resnet50()]
    raw = host_clients(entries, 5, seed=11, round_idx=1)
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    exp = orc.agg(args, copy.deepcopy(raw))
    res = ao.FedMLAggOperator.agg(args, _to_device(raw, cuda_device))
    for k in exp:
        assert res[k].dtype == exp[k].dtype, k
        gu.assert_same(res[k].cpu(), exp[k], k)


def test_native_walker_takes_device_dicts(cuda_device):
    """Device-resident dicts go through the native walker's pointer tables;
    anything irregular (here a non-contiguous client tensor) falls back to the
    Python walk, with the same result."""
    from fedml_amd import _native as nat

    w = ao._walker()
    assert w is not None
    entries = shapes.resnet50()
    raw = _to_device(host_clients(entries, 3, seed=2, round_idx=1), cuda_device)
    walked = w.walk([d for _, d in raw], list(raw[0][1].keys()))
    assert walked is not None
    dev, codes, numels, tables = walked
    assert dev == cuda_device.index or dev == 0
    assert set(tables) == {nat.DT_F32, nat.DT_I64}
    assert len(tables[nat.DT_F32]) == 8 * 3 * codes.count(nat.DT_F32)
    assert numels == [int(torch.Size(s).numel()) for _, s, _ in entries]
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    exp = orc.agg(args, [(n, OrderedDict((k, t.cpu()) for k, t in d.items())) for n, d in raw])
    k = "fc.weight"
    t = raw[1][1][k]
    raw[1][1][k] = t.t().contiguous().t()  # same values, not contiguous
    assert w.walk([d for _, d in raw], list(raw[0][1].keys())) is None
    res = ao.FedMLAggOperator.agg(args, raw)
    for key in exp:
        gu.assert_same(res[key].cpu(), exp[key], key)


def test_native_walker_allocates_outputs(cuda_device):
    """walk(..., alloc=True): one output per key, client 0's shape, float32 for
    int64 keys, on the inputs' device, and the output pointer tables match."""
    import numpy as np

    from fedml_amd import _native as nat

    w = ao._walker()
    entries = shapes.resnet50()[:12]
    raw = _to_device(host_clients(entries, 2, seed=4, round_idx=1), cuda_device)
    keys = list(raw[0][1].keys())
    dev, codes, numels, tables, outs, out_tables = w.walk([d for _, d in raw], keys, True)
    assert len(outs) == len(keys)
    for k, c, o in zip(keys, codes, outs):
        t0 = raw[0][1][k]
        assert o.shape == t0.shape and o.is_cuda and o.device == t0.device and o.is_contiguous()
        assert o.dtype == (torch.float32 if c == nat.DT_I64 else t0.dtype)
    for c, tab in out_tables.items():
        ptrs = np.frombuffer(tab, dtype=np.int64).tolist()
        assert ptrs == [o.data_ptr() for o, cc in zip(outs, codes) if cc == c]


def test_pipelined_walk_declines_in_a_later_chunk(cuda_device):
    """A small key (walked in the last chunk, after larger keys were already
    launched) that the walker declines: the general path recomputes every key
    and the result is still the reference's."""
    w = ao._walker()
    entries = shapes.resnet50()
    raw = _to_device(host_clients(entries, 3, seed=6, round_idx=2), cuda_device)
    keys = list(raw[0][1].keys())
    order = w.order_by_size(raw[0][1], keys)
    small = keys[order[-1]]
    assert order.index(keys.index(small)) >= sum(ao._CHUNK_KEYS)  # not in the first chunks
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    exp = orc.agg(args, [(n, OrderedDict((k, t.cpu()) for k, t in d.items())) for n, d in raw])
    t = raw[2][1][small]
    raw[2][1][small] = torch.empty(t.numel() * 2 + 2, dtype=t.dtype, device=t.device)[1::2][:t.numel()].view(t.shape)
    raw[2][1][small].copy_(t)
    res = ao.FedMLAggOperator.agg(args, raw)
    for key in exp:
        gu.assert_same(res[key].cpu(), exp[key], key)


def test_tail_chunks_on_side_stream_are_stream_ordered(cuda_device):
    """The small-key chunks launch on a side stream.  Called on a non-default
    stream whose queue still holds the inputs' producer (a slow GEMM chain
    feeding every client tensor), agg() must read the produced values, and the
    caller's stream must see the side stream's outputs without a device sync."""
    entries = shapes.resnet50()
    K = 4
    raw = host_clients(entries, K, seed=11, round_idx=3)
    keys = list(raw[0][1].keys())
    assert len(keys) > sum(ao._CHUNK_KEYS)  # some chunks go to the side stream
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    exp = orc.agg(args, copy.deepcopy(raw))
    staged = _to_device(raw, cuda_device)
    s = torch.cuda.Stream(cuda_device)
    torch.cuda.synchronize(cuda_device)
    with torch.cuda.stream(s):
        m = torch.randn(4096, 4096, device=cuda_device)
        for _ in range(8):  # tens of ms of queued work before the inputs exist
            m = torch.tanh(m @ m)
        one = (m[0, 0] * 0).abs() + 1  # 1, but only once the chain has run
        # the producers: x * 1 == x exactly, ordered after the GEMM chain on s
        dev = [(n, OrderedDict((k, x * one.to(x.dtype)) for k, x in d.items())) for n, d in staged]
        res = ao.FedMLAggOperator.agg(args, dev)
        got = OrderedDict((k, v.to("cpu", non_blocking=False)) for k, v in res.items())
    for key in exp:
        gu.assert_same(got[key], exp[key], key)


def test_unaligned_views_take_scalar_path(cuda_device):
    """Tensors that are views at odd element offsets (not 16-byte aligned)."""
    K, N = 5, 4099
    base = [torch.randn(N + 3, device=cuda_device) for _ in range(K)]
    views = [b[1:N + 1] for b in base]
    ns = [3, 1, 4, 1, 5]
    raw = [(n, OrderedDict(x=v)) for n, v in zip(ns, views)]
    res = ao.FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), raw)
    exp = orc.wsum([v.cpu() for v in views], [n / sum(ns) for n in ns])
    gu.assert_same(res["x"].cpu(), exp, "x")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_headline_shape_sampled_columns(dtype, cuda_device):
    """Config 3 at full size (128 x 25,610,152 fp32; bf16 for the config-4
    dtype): the kernel reduces every column independently, so the oracle is
    evaluated on 200,000 random columns (all 128 clients each) plus the ragged
    tail, and must match bit for bit."""
    K, N = 128, 25_610_152
    g = torch.Generator(device=cuda_device).manual_seed(7)
    rows = torch.empty((K, (N + 63) // 64 * 64), dtype=dtype, device=cuda_device)
    for i in range(K):
        rows[i].copy_(torch.randn(rows.shape[1], generator=g, device=cuda_device) * 0.05)
    ns = [int(v) for v in np.random.default_rng(3).integers(100, 1001, K)]
    ws = [n / sum(ns) for n in ns]
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    kn.wsum_tensors([rows[i, :N] for i in range(K)], ws, out)
    idx = torch.cat([torch.randint(0, N, (200_000,), generator=torch.Generator().manual_seed(1)),
                     torch.arange(N - 64, N)]).to(cuda_device)
    cols = rows[:, idx].cpu()
    exp = orc.wsum([cols[i] for i in range(K)], ws)
    gu.assert_same(out[idx].cpu(), exp, f"headline {dtype}")


@pytest.mark.parametrize("dtype,N", [(torch.float32, 4_194_305), (torch.float32, 16_777_216),
                                     (torch.bfloat16, 8_388_613), (torch.float16, 8_390_000),
                                     (torch.bfloat16, 8_388_607), (torch.float16, 1_000_003),
                                     (torch.float32, 1_048_575)])
def test_mid_size_tiles_vs_oracle(dtype, N, cuda_device):
    """Launches of 1,025..4,096 tiles take the one-client-per-step tile
    configuration (MidCfg); every element checked against the oracle,
    including the ragged tail."""
    K = 9
    g = torch.Generator(device=cuda_device).manual_seed(N % 1000)
    rows = (torch.randn((K, N), generator=g, device=cuda_device) * 0.05).to(dtype)
    ns = [int(v) for v in np.random.default_rng(N % 97).integers(100, 1001, K)]
    ws = [n / sum(ns) for n in ns]
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    kn.wsum_tensors([rows[i] for i in range(K)], ws, out)
    host = rows.cpu()
    exp = orc.wsum([host[i] for i in range(K)], ws)
    gu.assert_same(out.cpu(), exp, f"mid {dtype} {N}")


def test_bf16_fp32_accumulate_tolerance(cuda_device):
    """fedagg_low_precision_acc='fp32': within one bf16 rounding of the exact
    (fp64) weighted mean, |err| <= 2^-8 * |Σ w_i p_i| + 2^-133 (one final RNE)."""
    raw = host_clients([("h", (512 * 1024 + 5,), torch.bfloat16)], 64, seed=9)
    ns = [n for n, _ in raw]
    ws = [n / sum(ns) for n in ns]
    args = type("A", (), {"federated_optimizer": "FedAvg", "fedagg_low_precision_acc": "fp32"})()
    res = ao.FedMLAggOperator.agg(args, _to_device(raw, cuda_device))["h"].float().cpu().double()
    exact = sum(d["h"].double() * w for (_, d), w in zip(raw, ws))
    err = (res - exact).abs()
    bound = exact.abs() * 2.0 ** -8 + 1e-38
    assert bool((err <= bound).all()), float((err - bound).max())
    # and the reference chain (default) is much noisier at K=64
    ref_chain = ao.FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg"})(),
                                        _to_device(raw, cuda_device))["h"].float().cpu().double()
    assert float((ref_chain - exact).abs().mean()) > float(err.mean())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K,N", [(3, 1023), (48, 70_001), (600, 40_001), (600, 300_001), (9, 1_000_001)])
def test_fp32_accumulate_narrow_packs_vs_oracle(K, N, dtype, cuda_device):
    """fp32-accumulate mode on the narrow-pack tiles (16-bit rows below 8M
    elements), bit for bit against the oracle's fp32 chain with one final RNE,
    aligned and at a one-element offset."""
    g = torch.Generator(device=cuda_device).manual_seed(K + N)
    rows = (torch.randn((K, N + 1), generator=g, device=cuda_device) * 0.05).to(dtype)
    ns = [5 + 3 * i for i in range(K)]
    w = [n / sum(ns) for n in ns]
    for group in ([rows[i, :N] for i in range(K)], [rows[i, 1:] for i in range(K)]):
        out = torch.empty(N, device=cuda_device, dtype=dtype)
        kn.wsum_tensors(group, w, out, kn.ACC_FP32)
        exp = orc.wsum_acc32([t.cpu() for t in group], w)
        gu.assert_same(out.cpu(), exp, f"acc32 K={K} N={N} {dtype}")


def test_fedavg_seq_inplace_on_device(cuda_device):
    raw = host_clients([("w", (10001,), torch.float32), ("n", (3,), torch.int64), ("h", (777,), torch.bfloat16)],
                       6, seed=11)
    exp = orc.agg(type("A", (), {"federated_optimizer": "FedAvg_seq"})(), copy.deepcopy(raw))
    draw = _to_device(raw, cuda_device)
    t0 = dict(draw[0][1])
    res = ao.FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg_seq"})(), draw)
    for k in exp:
        assert res[k] is t0[k]
        gu.assert_same(res[k].cpu(), exp[k], k)


def test_kernel_errors_are_loud(cuda_device):
    from fedml_amd import _native as nat

    with pytest.raises(nat.FedAggNativeError):
        nat.check(nat.lib().fedagg_wsum_f32(None, None, 0, 10, None, 0, None), "bad")
    assert "K must be" in nat.lib().fedagg_last_error().decode()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64])
def test_client_axis_single_rank_kernel_path(dtype, cuda_device):
    """ClientAxisAggregator on one GPU (no collective): chunked kernel launches
    over pointer tables offset per chunk must reproduce the single chain
    (fp32 partial; bf16/int64 sources accumulate in fp32)."""
    from fedml_amd.sharded import ClientAxisAggregator

    K, L = 12, 300_007
    g = torch.Generator(device=cuda_device).manual_seed(4)
    rows = torch.zeros(K, (L + 63) // 64 * 64, device=cuda_device, dtype=dtype)
    if dtype == torch.int64:
        rows[:, :L] = torch.randint(-1000, 1000, (K, L), generator=g, device=cuda_device)
    else:
        rows[:, :L] = (torch.randn(K, L, generator=g, device=cuda_device) * 0.05).to(dtype)
    ns = list(range(10, 10 + K))
    ws = [n / sum(ns) for n in ns]
    agg = ClientAxisAggregator(rows, L, chunks=5)
    full = agg.aggregate(ws)[:L].cpu()
    cpu_rows = rows[:, :L].cpu()
    if dtype == torch.bfloat16:  # fp32 accumulate of bf16 inputs
        exp = orc.wsum([cpu_rows[i].float() for i in range(K)], ws)
    else:
        exp = orc.wsum([cpu_rows[i] for i in range(K)], ws)
    gu.assert_same(full, exp, f"client-axis {dtype}")


@pytest.mark.parametrize("K", [1, 7, 256, 257])
def test_kernel_argument_weights_match_device_weights(K, cuda_device):
    """FEDAGG_HOST_WEIGHTS (weights by value in the launch, K <= 256) and the
    device-array path give identical bits; K = 257 falls back to the array."""
    N = 70_001
    g = torch.Generator(device=cuda_device).manual_seed(K)
    rows = torch.randn(K, (N + 63) // 64 * 64, generator=g, device=cuda_device)
    ws = [float(i + 1) for i in range(K)]
    ws = [w / sum(ws) for w in ws]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    a = torch.empty(N, device=cuda_device)
    b = torch.empty(N, device=cuda_device)
    kn.wsum_ptrs(torch.float32, d_ptrs, kn.upload_f32(ws, cuda_device), K, N, a, True)
    hw = kn.weights_for(ws, torch.float32, cuda_device)
    assert isinstance(hw, kn.HostWeights) == (K <= 256)
    kn.wsum_ptrs(torch.float32, d_ptrs, hw, K, N, b, True)
    gu.assert_same(a.cpu(), b.cpu(), f"K={K}")
    exp = orc.wsum([rows[i, :N].cpu() for i in range(K)], ws)
    gu.assert_same(b.cpu(), exp, f"K={K} vs oracle")


@pytest.mark.parametrize("name", ["resnet_mini_k5", "resnet_mini_bigint_k3", "mixed_dtypes_k4"])
def test_bucket_device_inputs_int_promotion(name, cuda_device):
    """Integer keys ride in the fp32 rows as fl32(v) (converted on the GPU at
    ingest): bit-identical to the reference's int64 * w, also for |v| > 2^24."""
    meta, arrays = gu.load(name)
    raw = _to_device(cases.build_inputs(meta["spec"]), cuda_device)
    bucket = ClientBucket(raw[0][1], len(raw), cuda_device)
    assert all(k in bucket.int_keys for k, t in raw[0][1].items() if not t.is_floating_point())
    assert torch.int64 not in bucket.groups
    for i, (n, d) in enumerate(raw):
        bucket.put(i, d, n)
    res = bucket.aggregate()
    for k, e in gu.expected_groups(meta, arrays)[0].items():
        gu.assert_same(res[k].cpu(), e, f"{name}[{k}]")


@pytest.mark.parametrize("name", ["cfg2_cnn_web_k32", "resnet_mini_bigint_k3", "mixed_dtypes_k4", "ragged_f32_k17"])
@pytest.mark.parametrize("pinned", [False, True])
def test_put_encoded_matches_reference(name, pinned, cuda_device):
    """FAGG messages (fedml_amd.wire) ingested with one H2D per dtype group,
    from pageable or pinned receive buffers, aggregate to the reference bits."""
    from fedml_amd import wire

    meta, arrays = gu.load(name)
    raw = cases.build_inputs(meta["spec"])
    bucket = ClientBucket(raw[0][1], len(raw), cuda_device)
    msgs = []
    for n, d in raw:
        m = wire.encode(d, n)
        if pinned:
            t = torch.empty(len(m), dtype=torch.uint8).pin_memory()
            t.numpy()[:] = np.frombuffer(m, dtype=np.uint8)
            m = t.numpy()
        msgs.append(m)
    for i, m in enumerate(msgs):
        bucket.put_encoded(i, m)
    res = bucket.aggregate()
    for k, e in gu.expected_groups(meta, arrays)[0].items():
        gu.assert_same(res[k].cpu(), e, f"{name}[{k}]")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_round_f32_matches_torch_rounding(dtype, cuda_device):
    x = torch.randn(100_003, device=cuda_device) * 1e3
    x[:5] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e-40, -0.0])
    got = kn.round_f32(x, dtype).cpu()
    if dtype == torch.bfloat16:
        exp = torch.from_numpy(orc.f32_to_bf16_bits(x.cpu().numpy()).view(np.int16)).view(torch.bfloat16)
    else:
        exp = x.cpu().to(torch.float16)
    gu.assert_same(got, exp, str(dtype))



def test_small_host_rounds_take_the_batched_pack(cuda_device, monkeypatch):
    """Host dicts of a small round go through one pack + one H2D per dtype
    (bucket.put_batch), also with int64 counters promoted into the fp32 rows
    and across rounds that reuse the cached bucket's pinned staging; results
    stay bit-exact."""
    calls = []
    orig = ClientBucket.put_batch

    def spy(self, *a, **kw):
        calls.append(self.capacity)
        return orig(self, *a, **kw)

    monkeypatch.setattr(ClientBucket, "put_batch", spy)
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    entries = shapes.resnet50()[:24] + [("extra.f64", (5,), torch.float64), ("extra.bf16", (7, 3), torch.bfloat16)]
    for r in range(3):
        raw = host_clients(entries, 6, seed=40 + r, round_idx=r)
        exp = orc.agg(args, copy.deepcopy(raw))
        res = ao.FedMLAggOperator.agg(args, raw)
        for k in exp:
            assert not res[k].is_cuda and res[k].dtype == exp[k].dtype, k
            gu.assert_same(res[k], exp[k], f"round {r} {k}")
    assert calls == [6, 6, 6]


def test_large_host_rounds_stage_per_client_from_tables(cuda_device, monkeypatch):
    """Above the one-image limit, host rounds stage client by client from the
    walker's pointer tables (bucket.put_from_table), int64 counters included;
    bit-exact, and the cached bucket's ring is reused across rounds."""
    calls = []
    orig = ClientBucket.put_from_table

    def spy(self, slot, *a, **kw):
        calls.append(slot)
        return orig(self, slot, *a, **kw)

    monkeypatch.setattr(ClientBucket, "put_from_table", spy)
    monkeypatch.setattr(ao, "_BATCH_MAX_BYTES", 0)
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    entries = shapes.resnet50()[:40] + [("extra.f16", (9,), torch.float16)]
    for r in range(2):
        raw = host_clients(entries, 5, seed=60 + r, round_idx=r)
        exp = orc.agg(args, copy.deepcopy(raw))
        res = ao.FedMLAggOperator.agg(args, raw)
        for k in exp:
            assert not res[k].is_cuda and res[k].dtype == exp[k].dtype, k
            gu.assert_same(res[k], exp[k], f"round {r} {k}")
    assert calls == list(range(5)) * 2


def test_next_update_does_not_overtake_a_pending_reduction(cuda_device):
    """An update put() while the previous round's reduction is still queued on
    the caller's stream must not overwrite the rows under it: the reduction
    sees the old round, the next one the new data."""
    K, N = 3, 1 << 20
    bucket = ClientBucket([("x", (N,), torch.float32)], K, cuda_device)
    old = [torch.full((N,), float(i + 1)) for i in range(K)]
    new = torch.full((N,), 100.0)
    for i in range(K):
        bucket.put(i, {"x": old[i]}, 1)
    outs = bucket.new_outputs()
    w = bucket.weights([1, 1, 2])
    bucket.sync_ingest()
    torch.cuda._sleep(200_000_000)  # keep the stream busy so the reduction is still queued
    bucket.reduce_into(outs, w)
    bucket.put(0, {"x": new}, 1)  # host H2D on the copy stream
    first = outs[torch.float32][:N].clone()
    outs2 = bucket.new_outputs()
    bucket.reduce_into(outs2, w)
    torch.cuda.synchronize()
    exp_old = orc.wsum(old, w)
    exp_new = orc.wsum([new, old[1], old[2]], w)
    gu.assert_same(first.cpu(), exp_old, "pending reduction")
    gu.assert_same(outs2[torch.float32][:N].cpu(), exp_new, "next round")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [2, 17, 48, 100, 600])
@pytest.mark.parametrize("N", [1, 3, 5, 63, 65, 255, 257, 1023, 4_097, 40_001, 70_001])
def test_tight_tensors_every_tile_config(K, N, dtype, cuda_device):
    """Separately allocated client tensors of exactly N elements (no padding
    to read into), aligned and at an odd element offset, across the tile
    configs (narrow many-client packs, tiny, small, shipped) and their ragged
    edge paths; 16-bit rows on the reference chain."""
    g = torch.Generator(device=cuda_device).manual_seed(K * 100_003 + N)
    ts = [(torch.randn(N, generator=g, device=cuda_device) * 0.05).to(dtype) for _ in range(K)]
    views = [(torch.randn(N + 1, generator=g, device=cuda_device) * 0.05).to(dtype)[1:]
             for _ in range(K)]  # one-element offset: not 16-byte aligned
    ns = [3 + 7 * i for i in range(K)]
    w = [n / sum(ns) for n in ns]
    for group in (ts, views):
        out = torch.empty(N, device=cuda_device, dtype=dtype)
        kn.wsum_tensors(group, w, out)
        exp = orc.wsum([t.cpu() for t in group], w)
        gu.assert_same(out.cpu(), exp, f"K={K} N={N} {dtype}")


def test_put_interleaved_host_and_device_keys(cuda_device):
    """One dtype group holding host AND device keys in alternation: the host
    keys' staged H2D must not overwrite the device keys copied D2D between
    them (each stretch of host keys is its own copy).  Two rounds on the same
    slots, so stale staging bytes would show."""
    K = 3
    entries = [(f"k{j}", (n,), torch.float32) for j, n in enumerate([5, 70, 1, 64, 4099, 3, 129, 2])]
    bucket = ClientBucket(entries, K, cuda_device)
    for r in range(2):
        raw = host_clients(entries, K, seed=90 + r)
        exp = orc.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), copy.deepcopy(raw))
        for i, (n, d) in enumerate(raw):
            mixed = OrderedDict((k, t.to(cuda_device) if (j + i + r) % 2 else t) for j, (k, t) in enumerate(d.items()))
            bucket.put(i, mixed, n)
        res = bucket.aggregate()
        for k, e in exp.items():
            gu.assert_same(res[k].cpu(), e, f"round {r} {k}")


@pytest.mark.parametrize("model,K", [("lr_mnist", 4), ("cnn_web", 32), ("lr_mnist", 256), ("lr_mnist", 257),
                                     ("cnn_web", 1)])
def test_small_host_rounds_take_one_native_call(model, K, cuda_device, monkeypatch):
    """Configs 1 and 2 on host dicts: the whole round is fedagg_host_round_f32
    (zero-copy kernel at config 1's 125 KB, one DMA at config 2's 7.9 MB),
    bit-exact vs the oracle; results are new independent fp32 host tensors;
    K = 257 (beyond the inline weights) takes the staging path instead."""
    calls = []
    real = ao._reduce_host_round

    def spy(*a, **k):
        r = real(*a, **k)
        calls.append(r is not None)
        return r

    monkeypatch.setattr(ao, "_reduce_host_round", spy)
    raw = host_clients(shapes.MODELS[model](), K, seed=K)
    exp = orc.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), copy.deepcopy(raw))
    c0 = raw[0][1]
    res = ao.FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), raw)
    assert res is c0 and calls == [K <= 256]
    ptrs = set()
    for k, e in exp.items():
        assert not res[k].is_cuda and res[k].dtype == torch.float32 and res[k].is_contiguous()
        gu.assert_same(res[k], e, f"{model} K={K} {k}")
        ptrs.add(res[k].data_ptr())
    assert len(ptrs) == len(exp)


def test_host_round_mixed_int64_and_buffer_growth(cuda_device):
    """int64 keys enter as fl32(v) (|v| up to 2^40) with fp32 results, as
    the reference promotes them; consecutive rounds of different sizes
    (growing, then shrinking the library's pinned buffers) stay exact."""
    A = type("A", (), {"federated_optimizer": "FedAvg"})
    for name in ["resnet_mini_bigint_k3", "cfg2_cnn_web_k32", "cfg1_lr_mnist_k4", "resnet_mini_k5"]:
        meta, arrays = gu.load(name)
        raw = cases.build_inputs(meta["spec"])
        res = ao.FedMLAggOperator.agg(A(), raw)
        gu.assert_groups(res, meta, arrays, name)
