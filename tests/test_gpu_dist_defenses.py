"""GPU parity of the distance-based defenses (csrc/robust.hip) against the
reference's own KrumDefense / NormDiffClippingDefense outputs (tests/golden)
and against the numpy oracle; tolerances as stated in test_dist_defenses.py:
Krum's selection equals the reference's (tied fp32 scores excepted), the
aggregate after it is bit-exact; clipped weights within 2^-21 (|w| + |g|),
unclipped ones bit for bit.  Kernel level: dist2 (fp64 sums of exact squares)
within 1e-12 relative of numpy's fp64 sum, pairdist2 (fp32 stage sums) within
1e-5 relative, and the two kernels agree with each other at full size."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import _native as nat
from fedml_amd import defense as dfn
from fedml_amd import kernels as kn
from fedml_amd.server_aggregator import MI355XServerAggregator
from oracle import fedavg_oracle as orc
from test_dist_defenses import _m, assert_selection

pytestmark = pytest.mark.gpu

KRUM = [c["name"] for c in cases.DIST_CASES if c["defense"] in ("krum", "multikrum")]
CLIP = [c["name"] for c in cases.DIST_CASES if c["defense"] == "norm_diff_clipping"]


class _Agg(MI355XServerAggregator):
    def __init__(self, args, global_model=None):
        super().__init__(torch.nn.Linear(1, 1), args)
        self._g = global_model

    def get_model_params(self):
        return self._g


def _to(raw, dev):
    return [(n, OrderedDict((k, t.to(dev)) for k, t in d.items())) for n, d in raw]


@pytest.mark.parametrize("method", ["gram", "exact"])
@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", KRUM)
def test_krum_matches_reference(name, device_inputs, method, cuda_device):
    """Both pair-distance kernels (the centred fp32-MFMA Gram, K <= 128, and
    the exact-difference VALU kernel) select what the reference selects."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    if method == "gram" and spec["K"] > dfn.GRAM_MAX_CLIENTS:
        pytest.skip("the Gram kernel holds at most 128 clients")
    raw, _ = cases.dist_inputs(spec)
    if device_inputs:
        raw = _to(raw, cuda_device)
    args = cases.DefenseArgs(spec)
    args.fedagg_pair_distance = method
    agg = _Agg(args)
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            agg.on_before_aggregation(raw)
        assert type(ei.value).__name__ == meta["error"]
        return
    lst, idxs = agg.on_before_aggregation(raw)
    assert idxs == list(range(len(raw)))
    assert len(lst) == _m(spec)
    sel = [next(i for i, item in enumerate(raw) if item is s) for s in lst]  # the original tuples
    if assert_selection(sel, meta, name):
        res = agg.on_after_aggregation(agg.aggregate(lst))
        for t in res.values():
            assert t.is_cuda == device_inputs
        gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", CLIP)
def test_clip_matches_reference(name, device_inputs, cuda_device):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, glob = cases.dist_inputs(spec)
    if device_inputs:
        raw, glob = _to(raw, cuda_device), OrderedDict((k, t.to(cuda_device)) for k, t in glob.items())
    agg = _Agg(cases.DefenseArgs(spec), glob)
    lst, _ = agg.on_before_aggregation(raw)
    assert len(lst) == len(raw)
    for i, (n, d) in enumerate(lst):
        assert n == raw[i][0]
        clipped = meta["ref_norms"][i] / spec["norm_bound"] > 1
        for k, t in d.items():
            if not dfn.is_weight_param(k):
                assert t is raw[i][1][k]  # the client's own tensor, as the reference keeps it
            assert t.is_cuda == device_inputs
            ref = arrays[f"c{i}:{k}"].reshape(-1)
            got = t.cpu().numpy().reshape(-1)
            if not clipped or not dfn.is_weight_param(k):
                np.testing.assert_array_equal(got.view(np.uint8), ref.view(np.uint8), err_msg=f"{name} c{i}:{k}")
            else:
                gk = glob[k].cpu().numpy().reshape(-1)
                assert (np.abs(got - ref) <= 2.0 ** -21 * (np.abs(ref) + np.abs(gk))).all(), f"{name} c{i}:{k}"
    res = agg.aggregate(lst)
    for k, t in res.items():
        np.testing.assert_allclose(t.cpu().numpy(), arrays[f"o0:{k}"], rtol=1e-5, atol=1e-7, err_msg=k)
    if not any(v / spec["norm_bound"] > 1 for v in meta["ref_norms"]):
        gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


def _rows(K, L, dev, seed, outliers=()):
    g = torch.Generator(device=dev).manual_seed(seed)
    base = torch.randn(L, generator=g, device=dev) * 0.05
    rows = base + 0.01 * torch.randn((K, L), generator=g, device=dev)
    for i in outliers:
        rows[i] *= 3.0
    return rows


def _chunks(segs, chunk, dev):
    tab = []
    for off, n in segs:
        for s in range(off, off + n, chunk):
            tab += [s, min(chunk, off + n - s)]
    return kn.upload_i64(tab, dev), len(tab) // 2


def _np_pair(rows_np, segs):
    cols = np.concatenate([np.arange(o, o + n) for o, n in segs])
    X = rows_np[:, cols]
    K = X.shape[0]
    D = np.zeros((K, K))
    for i in range(K):
        d = (X[i][None, :] - X).astype(np.float32).astype(np.float64)
        D[i] = (d * d).sum(axis=1)
    return D


@pytest.mark.parametrize("K", [1, 2, 3, 17, 63, 64, 65, 100, 128, 129, 200])
def test_pairdist2_vs_numpy(K, cuda_device):
    L = 5000
    rows = _rows(K, L, cuda_device, K, outliers=[0] if K > 2 else [])
    segs = [(0, 1), (3, 700), (704, 1), (960, 2500), (4000, 999)]  # ragged, partial stages
    chunks, n = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    D = dfn.pairdist2_rows(ptrs, K, chunks, n, cuda_device, "exact").cpu().numpy()
    want = _np_pair(rows.cpu().numpy(), segs)
    np.testing.assert_allclose(D, want, rtol=1e-5)
    assert (np.diag(D) == 0).all()
    np.testing.assert_array_equal(D, D.T)


# every group count NB = ceil(K / 16) of the split kernel's builds, 1 .. 8
# (33 / 48: NB = 3, 81 / 96: NB = 6), with both full and partial last groups
@pytest.mark.parametrize("K", [1, 2, 3, 16, 17, 33, 48, 63, 64, 65, 81, 96, 100, 127, 128])
def test_pairgram2_vs_numpy(K, cuda_device):
    """The centred Gram: every pair within 2e-6 of the exact fp32-difference
    distances relative to (|c_i|^2 + |c_j|^2) of the column-centred rows (and
    so, for these rows, within 1e-5 of D itself), symmetric, 0 on the
    diagonal, never negative."""
    L = 5000
    rows = _rows(K, L, cuda_device, 100 + K, outliers=[0] if K > 2 else [])
    segs = [(0, 1), (3, 700), (704, 1), (960, 2500), (4000, 999)]  # ragged, partial stages
    chunks, n = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    D = dfn.pairdist2_rows(ptrs, K, chunks, n, cuda_device, "gram").cpu().numpy()
    want = _np_pair(rows.cpu().numpy(), segs)
    cols = np.concatenate([np.arange(o, o + m) for o, m in segs])
    X = rows.cpu().numpy()[:, cols].astype(np.float64)
    C = X - X.mean(axis=0)[None, :]
    nrm = (C * C).sum(axis=1)
    scale = nrm[:, None] + nrm[None, :]
    assert (np.abs(D - want) <= 2e-6 * scale + 1e-300).all(), np.abs(D - want).max()
    np.testing.assert_allclose(D, want, rtol=1e-5)
    assert (np.diag(D) == 0).all() and (D >= 0).all()
    np.testing.assert_array_equal(D, D.T)


@pytest.mark.parametrize("scale", [1.0, 3.0, 1e3])
def test_auto_pair_distance_falls_back_for_a_far_outlier(scale, cuda_device):
    """Krum's default ("auto"): one client scaled far from the rest (the
    Byzantine update Krum exists for) moves the client mean, so the centred
    Gram's error on the honest pairs grows with that update's norm.  auto
    then returns the exact kernel's distances (bit for bit), and Krum selects
    what the exact kernel selects; near the cluster (scale 1 or 3) it keeps the
    Gram's distances."""
    K, L = 40, 200_000
    rows = _rows(K, L, cuda_device, 9)
    rows[7] *= scale
    segs = [(0, L)]
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    ch, n = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    Dg = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "gram").cpu().numpy()
    De = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "exact").cpu().numpy()
    Da = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "auto").cpu().numpy()
    cond = dfn.gram_condition(Dg)
    if scale >= 1e3:
        assert cond > 100 * dfn.GRAM_MAX_CONDITION
        np.testing.assert_array_equal(Da, De)
    else:
        assert cond < dfn.GRAM_MAX_CONDITION
        np.testing.assert_array_equal(Da, Dg)
    sa = torch.argsort(torch.Tensor(dfn.krum_scores(Da, 5))).tolist()
    se = torch.argsort(torch.Tensor(dfn.krum_scores(De, 5))).tolist()
    assert sa[:10] == se[:10]
    if scale > 1.0:
        assert 7 not in sa[:K - 5]


@pytest.mark.parametrize("bad", ["inf", "nan", "1e30"])
def test_auto_pair_distance_falls_back_for_a_non_finite_outlier(bad, cuda_device):
    """A client with an inf / NaN element, or scaled so far (1e30) that its
    fp32 squares overflow, makes the centred Gram non-finite.  auto must then
    hand the exact kernel's distances back (bit for bit, inf where the
    reference's torch.norm gives inf), and Krum keeps that client out, as the
    exact kernel and the reference do."""
    K, L = 24, 30_000
    rows = _rows(K, L, cuda_device, 11)
    if bad == "inf":
        rows[5, 123] = float("inf")
    elif bad == "nan":
        rows[5, 77] = float("nan")
    else:
        rows[5] *= 1e30
    segs = [(0, L)]
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    ch, n = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    Dg = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "gram").cpu().numpy()
    De = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "exact").cpu().numpy()
    Da = dfn.pairdist2_rows(ptrs, K, ch, n, cuda_device, "auto").cpu().numpy()
    assert dfn.gram_condition(Dg) == float("inf")
    np.testing.assert_array_equal(Da, De)
    if bad != "nan":
        sa = np.argsort(dfn.krum_scores(Da, 3), kind="stable").tolist()
        assert sa[-1] == 5 and 5 not in sa[:K - 3]


def test_gram_condition_non_finite_entries():
    D = np.ones((3, 3)) - np.eye(3)
    assert dfn.gram_condition(D) < dfn.GRAM_MAX_CONDITION
    for v in (float("inf"), float("nan")):
        E = D.copy()
        E[0, 1] = E[1, 0] = v
        assert dfn.gram_condition(E) == float("inf")


def test_pairgram2_rejects_more_than_128_clients(cuda_device):
    rows = _rows(129, 64, cuda_device, 1)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(129)], cuda_device)
    chunks, n = _chunks([(0, 64)], nat.PAIR_CHUNK, cuda_device)
    with pytest.raises(ValueError):
        dfn.pairdist2_rows(ptrs, 129, chunks, n, cuda_device, "gram")
    assert nat.lib().fedagg_robust_work_len(nat.WORK_PAIRGRAM, 129, 1) == -1


def test_full_size_gram_agrees_with_exact(cuda_device):
    """Config 3's size (128 clients x 25.6M columns, two outliers): the Gram
    matrix within 2e-6 relative of the exact-difference kernel's, and Krum's
    scores order the clients the same way."""
    K, L = 128, 25_610_240
    rows = _rows(K, L, cuda_device, 3, outliers=[5, 77])
    segs = [(0, 25_610_152)]
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    ch_p, n_p = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    Dg = dfn.pairdist2_rows(ptrs, K, ch_p, n_p, cuda_device, "gram").cpu().numpy()
    De = dfn.pairdist2_rows(ptrs, K, ch_p, n_p, cuda_device, "exact").cpu().numpy()
    np.testing.assert_allclose(Dg, De, rtol=2e-6)
    sg, se = dfn.krum_scores(Dg, 10), dfn.krum_scores(De, 10)
    og = torch.argsort(torch.Tensor(sg)).tolist()
    oe = torch.argsort(torch.Tensor(se)).tolist()
    assert og[:32] == oe[:32] and 5 not in og[:5] and 77 not in og[:5]


@pytest.mark.parametrize("with_ref", [False, True])
@pytest.mark.parametrize("K", [1, 5, 128, 300])
def test_dist2_vs_numpy(K, with_ref, cuda_device):
    L = 9000
    rows = _rows(K, L, cuda_device, 7 + K)
    ref = torch.randn(L, device=cuda_device) * 0.05 if with_ref else None
    segs = [(5, 2048), (2053, 1), (3000, 5999)]
    chunks, n = _chunks(segs, nat.DIST_CHUNK, cuda_device)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    got = dfn.dist2_rows(ptrs, K, ref, chunks, n, cuda_device).cpu().numpy()
    cols = np.concatenate([np.arange(o, o + m) for o, m in segs])
    X = rows.cpu().numpy()[:, cols]
    r = ref.cpu().numpy()[cols] if with_ref else np.zeros(len(cols), np.float32)
    d = (X - r[None, :]).astype(np.float32).astype(np.float64)
    np.testing.assert_allclose(got, (d * d).sum(axis=1), rtol=1e-12)


def test_empty_chunk_table(cuda_device):
    rows = _rows(3, 64, cuda_device, 1)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(3)], cuda_device)
    empty = torch.zeros(2, dtype=torch.int64, device=cuda_device)
    assert (dfn.pairdist2_rows(ptrs, 3, empty, 0, cuda_device, "exact") == 0).all()
    assert (dfn.pairdist2_rows(ptrs, 3, empty, 0, cuda_device, "gram") == 0).all()
    assert (dfn.dist2_rows(ptrs, 3, None, empty, 0, cuda_device) == 0).all()


def test_full_size_pairdist_agrees_with_dist2(cuda_device):
    """128 clients x 25.6M columns (config 3's row): sampled pairs of the
    packed-fp32 pair kernel against the fp64 single-reference kernel."""
    K, L = 128, 25_610_240
    rows = _rows(K, L, cuda_device, 3, outliers=[5, 77])
    segs = [(0, 25_610_152)]
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    ch_p, n_p = _chunks(segs, nat.PAIR_CHUNK, cuda_device)
    D = dfn.pairdist2_rows(ptrs, K, ch_p, n_p, cuda_device, "exact").cpu().numpy()
    ch_d, n_d = _chunks(segs, nat.DIST_CHUNK, cuda_device)
    for j in (0, 5, 64, 127):
        col = dfn.dist2_rows(ptrs, K, rows[j], ch_d, n_d, cuda_device).cpu().numpy()
        np.testing.assert_allclose(D[:, j], col, rtol=2e-6)
    # Krum at this size picks neither outlier
    scores = dfn.krum_scores(D, 10)
    best = torch.argsort(torch.Tensor(scores)).tolist()[:5]
    assert 5 not in best and 77 not in best


def test_clip_kernel_vs_oracle_large(cuda_device):
    K, L = 16, 1_000_064
    rows = _rows(K, L, cuda_device, 11, outliers=[3])
    g = torch.randn(L, device=cuda_device) * 0.05
    divs = [1.0, 1.5, 3.0000002, 1.0] * 4
    d_div = kn.upload_f32(divs, cuda_device)
    out = torch.empty_like(rows)
    ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    dst = kn.upload_i64([out[i].data_ptr() for i in range(K)], cuda_device)
    nat.check(nat.lib().fedagg_clip_diff_f32(ptrs.data_ptr(), K, g.data_ptr(), d_div.data_ptr(), L, dst.data_ptr(),
                                             nat.stream_handle()), "clip")
    x, gn = rows.cpu().numpy(), g.cpu().numpy()
    for i in range(K):
        want = (((x[i] - gn).astype(np.float32) / np.float32(divs[i])).astype(np.float32) + gn).astype(np.float32)
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.int32), want.view(np.int32))


def test_krum_on_bucket_views_cross_silo_style(cuda_device):
    """Device dicts that are views into one bucket (the cross-silo server's
    model_dict) with BatchNorm buffers among the keys: the chunk table skips
    the buffers, the result equals the oracle's selection."""
    spec = next(c for c in cases.DIST_CASES if c["name"] == "multikrum_dist_k70_m5")
    raw, _ = cases.dist_inputs(spec)
    from fedml_amd.bucket import ClientBucket

    b = ClientBucket(raw[0][1], len(raw), cuda_device, promote_ints=False)
    for i, (n, d) in enumerate(raw):
        b.put(i, d, n)
    b.sync_ingest()
    views = [(n, b.view(i)) for i, (n, _) in enumerate(raw)]
    got = dfn.krum_before_aggregation(views, spec["byzantine_client_num"], spec["krum_param_m"])
    want, _ = orc.krum_select(raw, spec["byzantine_client_num"], spec["krum_param_m"])
    pos = lambda lst, x: next(i for i, v in enumerate(lst) if v is x)  # noqa: E731
    assert [pos(views, x) for x in got] == [pos(raw, x) for x in want]


SLSGD = [c["name"] for c in cases.DIST_CASES if c["defense"] == "slsgd"]
CCLIP = [c["name"] for c in cases.DIST_CASES if c["defense"] == "cclip"]


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", SLSGD)
def test_slsgd_matches_reference(name, device_inputs, cuda_device):
    """SLSGD: trim by sample count, FedAvg, (1 - alpha) g + alpha avg on the GPU: bit for bit."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, glob = cases.dist_inputs(spec)
    if device_inputs:
        raw, glob = _to(raw, cuda_device), OrderedDict((k, t.to(cuda_device)) for k, t in glob.items())

    def run():
        agg = _Agg(cases.DefenseArgs(spec), glob)
        lst, _ = agg.on_before_aggregation(raw)
        return lst, agg.on_after_aggregation(agg.aggregate(lst))

    if meta["error"]:
        with pytest.raises(Exception) as ei:
            run()
        assert type(ei.value).__name__ == meta["error"]
        return
    lst, res = run()
    assert [next(i for i, it in enumerate(raw) if it[1] is x[1]) for x in lst] == meta["selected"]
    for t in res.values():
        assert t.is_cuda == device_inputs
    gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", CCLIP)
def test_cclip_matches_reference(name, device_inputs, cuda_device):
    """CClip: bucket means (our FedAvg kernel per group), the seeded guess,
    scaled differences, FedAvg, guess added back after aggregation."""
    from test_dist_defenses import assert_cclip_list, assert_close_groups

    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, _ = cases.dist_inputs(spec)
    if device_inputs:
        raw = _to(raw, cuda_device)
    agg = _Agg(cases.DefenseArgs(spec))
    np.random.seed(spec["np_seed"])
    lst, idxs = agg.on_before_aggregation(raw)
    assert idxs == list(range(len(raw)))
    assert [n for n, _ in lst] == meta["bucket_nums"]
    for _, d in lst:
        for t in d.values():
            assert t.is_cuda == device_inputs
    assert_cclip_list(lst, meta, arrays, name)
    res = agg.on_after_aggregation(agg.aggregate(lst))
    assert_close_groups(res, meta, arrays, name)


RLR = [c["name"] for c in cases.DIST_CASES if c["defense"] == "robust_learning_rate"]


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", RLR)
def test_robust_learning_rate_matches_reference(name, device_inputs, cuda_device):
    """RobustLearningRateDefense.run through the GPU drop-in (one fused pass:
    FedAvg chain + sign sum + the lr rule) vs the reference's own outputs, bit
    for bit; client 0's dict comes back with its keys rebound, on the inputs'
    device; threshold 0 goes to the base function (here our FedAvg)."""
    from fedml_amd.agg_operator import FedMLAggOperator

    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, _ = cases.dist_inputs(spec)
    if device_inputs:
        raw = _to(raw, cuda_device)
    args = cases.DefenseArgs(spec)
    d = dfn.RobustLearningRateDefense(args)
    res = d.run(raw, lambda lst: FedMLAggOperator.agg(args, lst))
    assert (res is raw[0][1]) == meta["returns_client0_dict"]
    for t in res.values():
        assert t.is_cuda == device_inputs
    gu.assert_groups(OrderedDict((k, t.cpu()) for k, t in res.items()), meta, arrays, name)


def test_robust_learning_rate_plugin_path_is_plain_fedavg(cuda_device):
    """As in FedML, "robust_learning_rate" is not one of FedMLDefender's
    before / on / after hooks: the plugin path aggregates plain FedAvg."""
    spec = next(c for c in cases.DIST_CASES if c["name"] == "rlr_resnet_mini_k8_t4")
    raw, _ = cases.dist_inputs(spec)
    args = cases.DefenseArgs(spec)
    agg = _Agg(args)
    lst, idxs = agg.on_before_aggregation(cases.clone_raw(raw))
    assert idxs == list(range(len(raw)))
    res = agg.on_after_aggregation(agg.aggregate(lst))
    want = orc.agg(args, cases.clone_raw(raw))
    for k in want:
        gu.assert_same(res[k].cpu(), want[k], k)


@pytest.mark.parametrize("K,N", [(3, 1), (7, 4099), (128, 1_000_003), (300, 65_537)])
def test_robust_learning_rate_kernel_vs_oracle(K, N, cuda_device):
    """The fused kernel on bucket-shaped rows vs the oracle: ragged N (edge
    path), K above the 256 inline weights (device weight array), sign-split,
    zero and NaN / inf coordinates, thresholds that flip some coordinates."""
    g = torch.Generator().manual_seed(K + N)
    base = torch.randn(N, generator=g)
    rows = [base + 0.5 * torch.randn(N, generator=g) for _ in range(K)]
    for r in rows[: K // 3]:
        r.neg_()
    rows[0][: min(N, 5)] = 0.0
    if N > 20:
        rows[K // 2][10] = float("nan")
        rows[-1][11] = float("inf")
        rows[1 % K][12] = -float("inf")
    raw = [(float(10 + i % 7), OrderedDict(x=r.clone())) for i, r in enumerate(rows)]
    thr = max(1, K // 3)
    want = orc.robust_learning_rate([(n, OrderedDict(x=d["x"].clone())) for n, d in raw], thr)["x"]
    dev_raw = _to(raw, cuda_device)
    got = dfn.robust_learning_rate(dev_raw, thr)["x"]
    gu.assert_same(got.cpu(), want, f"rlr K={K} N={N}")
