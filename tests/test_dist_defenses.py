"""Distance-based defenses (Krum / multi-Krum, norm-diff clipping, CClip) and
SLSGD, CPU side:
the oracle against the reference's own outputs (tests/golden, made by running
KrumDefense / NormDiffClippingDefense + FedMLAggOperator.agg), the chunk-table
builder, and the C ABI's argument checks (no GPU needed).

Tolerances, stated once: the reference takes an fp32 torch.norm of the fp32
difference vector; the oracle (and the kernels) sum the exact squares of the
same fp32 differences in fp64 and round the root to fp32.  Krum scores agree
to 1e-6 relative; the selection is the reference's exactly unless two fp32
scores tie within that (mirror-image clients of the fake model list); a
clipping divisor can differ in its last bit, so clipped weights agree to
2^-21 (|w| + |g|) per element (the divisor moves the quotient by an ulp
before the add), unclipped ones bit for bit.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import _native as nat
from fedml_amd import defense as dfn
from fedml_amd.layout import RowLayout
from fedml_amd.synth import fingerprint
from oracle import fedavg_oracle as orc

DIST = [c["name"] for c in cases.DIST_CASES]
SLSGD = [c["name"] for c in cases.DIST_CASES if c["defense"] == "slsgd"]
CCLIP = [c["name"] for c in cases.DIST_CASES if c["defense"] == "cclip"]
KRUM = [c["name"] for c in cases.DIST_CASES if c["defense"] in ("krum", "multikrum")]
CLIP = [c["name"] for c in cases.DIST_CASES if c["defense"] == "norm_diff_clipping"]
RLR = [c["name"] for c in cases.DIST_CASES if c["defense"] == "robust_learning_rate"]


def _m(spec):
    m = spec.get("krum_param_m")
    return m if isinstance(m, int) else 1


def assert_selection(sel, meta, what=""):
    """Same clients as the reference's, or tied ones (by the reference's own scores)."""
    ref_sel = meta["selected"]
    if list(sel) == list(ref_sel):
        return True
    rs = np.asarray(meta["ref_scores"])
    np.testing.assert_allclose(np.sort(rs[list(sel)]), np.sort(rs[list(ref_sel)]), rtol=1e-6, err_msg=what)
    return False


@pytest.mark.parametrize("name", DIST)
def test_inputs_reproducible(name):
    meta, _ = gu.load(name)
    raw, _ = cases.dist_inputs(meta["spec"])
    assert fingerprint(raw) == meta["in_sha256"]


@pytest.mark.parametrize("name", KRUM)
def test_oracle_krum_matches_reference(name):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, _ = cases.dist_inputs(spec)
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            orc.krum_select(raw, spec["byzantine_client_num"], _m(spec))
        assert type(ei.value).__name__ == meta["error"]
        return
    sel, scores = orc.krum_select(raw, spec["byzantine_client_num"], _m(spec))
    np.testing.assert_allclose(scores, meta["ref_scores"], rtol=1e-6)
    idx = [next(i for i, item in enumerate(raw) if item is s) for s in sel]
    if assert_selection(idx, meta, name):
        gu.assert_groups(orc.agg(cases.DefenseArgs(spec), sel), meta, arrays, name)


def test_krum_fake_list_tie_is_real():
    """The reference test's model list (clients i * A) has mirror-image
    clients whose scores tie: the tolerance above is about them."""
    meta, _ = gu.load("krum_fake_k20")
    s = np.asarray(meta["ref_scores"])
    i, j = 8, 9  # clients 9 and 10 of 20
    assert abs(s[i] - s[j]) <= 1e-6 * s[i]


@pytest.mark.parametrize("name", CLIP)
def test_oracle_clip_matches_reference(name):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, glob = cases.dist_inputs(spec)
    out = orc.norm_diff_clip(raw, glob, spec["norm_bound"])
    for i, (n, d) in enumerate(out):
        clipped = meta["ref_norms"][i] / spec["norm_bound"] > 1
        for k, t in d.items():
            ref = arrays[f"c{i}:{k}"].reshape(-1)
            got = t.numpy().reshape(-1)
            if not clipped or not orc._is_weight_param(k):
                np.testing.assert_array_equal(got.view(np.uint8), ref.view(np.uint8), err_msg=f"{name} c{i}:{k}")
            else:
                # divisors one ulp apart: |d/c| moves by <= 1.5 ulp, then + g rounds
                gk = glob[k].numpy().reshape(-1)
                tol = 2.0 ** -21 * (np.abs(ref) + np.abs(gk))
                assert (np.abs(got - ref) <= tol).all(), f"{name} c{i}:{k}"
    res = orc.agg(cases.DefenseArgs(spec), out)
    for k, t in res.items():
        np.testing.assert_allclose(t.numpy(), arrays[f"o0:{k}"], rtol=1e-5, atol=1e-7, err_msg=f"{name} {k}")
    if not any(v / spec["norm_bound"] > 1 for v in meta["ref_norms"]):
        gu.assert_groups(res, meta, arrays, name)  # nothing clipped: bit for bit


def test_ref_norms_match_oracle_fp32_root():
    for name in CLIP:
        meta, _ = gu.load(name)
        raw, glob = cases.dist_inputs(meta["spec"])
        g = orc.weight_vector(glob)
        ours = [orc.fp32_norm(orc.dist2(orc.weight_vector(p), g)) for _, p in raw]
        np.testing.assert_allclose(ours, meta["ref_norms"], rtol=4e-7)  # torch's fp32 sum: within 2 ulp


def test_weight_chunks_skip_buffers_and_split():
    layout = RowLayout([("conv.weight", (3, 5000), torch.float32), ("bn.weight", (7,), torch.float32),
                        ("bn.running_mean", (7,), torch.float32), ("bn.num_batches_tracked", (), torch.int64),
                        ("fc.weight", (4097,), torch.float32)], True)
    g = layout.groups[torch.float32]
    tab, n = dfn.weight_chunks(g, 2048, torch.device("cpu"), absolute=False)
    t = tab.view(-1, 2).numpy()
    assert n == len(t)
    cols = np.concatenate([np.arange(s, s + l) for s, l in t])
    want = np.concatenate([np.arange(o, o + m) for k, o, m in zip(g.keys, g.offsets, g.numels)
                           if dfn.is_weight_param(k)])
    np.testing.assert_array_equal(cols, want)
    assert (t[:, 1] <= 2048).all() and (t[:, 1] > 0).all()


@pytest.mark.parametrize("chunk", [8, 64, 2048])
def test_weight_chunks_absolute_cuts(chunk):
    """The default table: the same columns, cut at multiples of `chunk` in the row
    (only a run's first piece may start elsewhere), in order, none empty."""
    layout = RowLayout([("a.weight", (3, 501), torch.float32), ("bn.weight", (7,), torch.float32),
                        ("bn.running_mean", (7,), torch.float32), ("bn.num_batches_tracked", (), torch.int64),
                        ("fc.weight", (4097,), torch.float32), ("fc.bias", (5,), torch.float32)], True)
    g = layout.groups[torch.float32]
    t = dfn.weight_chunks(g, chunk, torch.device("cpu"))[0].view(-1, 2).numpy()
    cols = np.concatenate([np.arange(s, s + l) for s, l in t])
    want = np.concatenate([np.arange(o, o + m) for k, o, m in zip(g.keys, g.offsets, g.numels)
                           if dfn.is_weight_param(k)])
    np.testing.assert_array_equal(cols, want)
    assert (t[:, 1] > 0).all() and (t[:, 1] <= chunk).all()
    run_first = np.r_[True, t[1:, 0] != t[:-1, 0] + t[:-1, 1]]
    assert (t[~run_first, 0] % chunk == 0).all()
    # a piece never crosses a multiple of chunk
    assert ((t[:, 0] // chunk) == ((t[:, 0] + t[:, 1] - 1) // chunk)).all()


def test_abi_argument_checks():
    fbuild = pytest.importorskip("fedml_amd.build")
    fbuild.build()
    lib = nat.lib()
    assert lib.fedagg_robust_work_len(nat.WORK_DIST2, 0, 5) == -1
    assert lib.fedagg_robust_work_len(nat.WORK_PAIRDIST2, 130, 0) == 0
    assert lib.fedagg_robust_work_len(nat.WORK_PAIRDIST2, 130, 10) >= 6 * 64 * 64
    # up to 128 clients the triangle kernel: 16 slots per 4x4 pair block of the
    # upper triangle, one set per chunk group (at most one group per chunk)
    assert lib.fedagg_robust_work_len(nat.WORK_PAIRDIST2, 128, 10) == 16 * 528 * 10
    assert lib.fedagg_robust_work_len(nat.WORK_PAIRDIST2, 64, 3) == 16 * 136 * 3
    assert lib.fedagg_robust_work_len(nat.WORK_PAIRDIST2, 5, 1) == 16 * 3
    assert lib.fedagg_robust_work_len(7, 4, 4) == -1
    assert lib.fedagg_dist2_f32(None, 0, None, None, 0, None, None, 0, None) == -1
    assert b"K must be" in lib.fedagg_last_error()
    assert lib.fedagg_pairdist2_f32(1, 4, None, 3, 1, None, 0, None) == -1
    assert b"null pointer" in lib.fedagg_last_error()
    assert lib.fedagg_clip_diff_f32(1, 2, 1, 1, -1, 1, None) == -1


def test_krum_argument_error_before_any_device_work():
    raw, _ = cases.dist_inputs(next(c for c in cases.DIST_CASES if c["name"] == "krum_bad_f"))
    with pytest.raises(ValueError):
        dfn.krum_before_aggregation(raw, 2, 1)


@pytest.mark.parametrize("name", SLSGD)
def test_oracle_slsgd_matches_reference(name):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, glob = cases.dist_inputs(spec)
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            orc.slsgd(cases.DefenseArgs(spec), raw, glob)
        assert type(ei.value).__name__ == meta["error"]
        return
    res, lst = orc.slsgd(cases.DefenseArgs(spec), raw, glob)
    assert [next(i for i, it in enumerate(raw) if it[1] is x[1]) for x in lst] == meta["selected"]
    gu.assert_groups(res, meta, arrays, name)  # bit for bit


@pytest.mark.parametrize("name", CCLIP)
def test_oracle_cclip_matches_reference(name):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, _ = cases.dist_inputs(spec)
    np.random.seed(spec["np_seed"])
    new, guess = orc.cclip(raw, cases.DefenseArgs(spec).__dict__.get("tau", 10), spec["bucket_size"])
    assert [n for n, _ in new] == meta["bucket_nums"]
    assert_cclip_list(new, meta, arrays, name)
    res = orc.cclip_after(orc.agg(cases.DefenseArgs(spec), new), guess)
    assert_close_groups(res, meta, arrays, name)


def assert_cclip_list(new, meta, arrays, name):
    """CClip's scaled differences: bit for bit where the score is 1 (the guess's
    own bucket, and buckets within tau); a score below 1 comes from the fp32
    norm (within 2 ulp of torch's), so those agree to 2^-21 relative."""
    for b, (_, d) in enumerate(new):
        for k, t in d.items():
            got = t.cpu().numpy().reshape(-1)
            ref = arrays[f"c{b}:{k}"].reshape(-1)
            if not np.array_equal(got.view(np.uint32), ref.view(np.uint32)):
                assert (np.abs(got - ref) <= 2.0 ** -21 * np.abs(ref)).all(), f"{name} c{b}:{k}"


def assert_close_groups(res, meta, arrays, name):
    for k, t in res.items():
        np.testing.assert_allclose(t.cpu().numpy().reshape(-1), arrays[f"o0:{k}"].reshape(-1), rtol=1e-5, atol=1e-6,
                                   err_msg=f"{name} {k}")


@pytest.mark.parametrize("name", RLR)
def test_oracle_robust_learning_rate_matches_reference(name):
    """RobustLearningRateDefense.run restated (oracle) vs the reference's own
    outputs, bit for bit; client 0's dict is the returned object."""
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw, _ = cases.dist_inputs(spec)
    args = cases.DefenseArgs(spec)
    res = orc.robust_learning_rate(raw, spec["robust_threshold"], lambda lst: orc.agg(args, lst))
    assert (res is raw[0][1]) == meta["returns_client0_dict"]
    gu.assert_groups(res, meta, arrays, name)


def test_oracle_robust_learning_rate_signs():
    """The lr rule on a hand case: 3 clients, threshold 2 -> coordinates whose
    signs agree keep the average, split or zero ones flip it, NaN stays NaN."""
    t = [torch.tensor([1.0, 2.0, -1.0, 0.0, float("nan")]), torch.tensor([3.0, -2.0, -1.0, 0.0, 1.0]),
         torch.tensor([2.0, 1.0, -4.0, 0.0, 1.0])]
    raw = [(1, OrderedDict(x=t[0].clone())), (1, OrderedDict(x=t[1].clone())), (2, OrderedDict(x=t[2].clone()))]
    out = orc.robust_learning_rate(raw, 2)["x"].numpy()
    w = [np.float32(0.25), np.float32(0.25), np.float32(0.5)]
    avg = (t[0].numpy() * w[0] + t[1].numpy() * w[1]) + t[2].numpy() * w[2]
    assert out[0] == avg[0] and out[2] == avg[2]  # |3| >= 2
    assert out[1] == -avg[1]  # |1 - 1 + 1| = 1 < 2
    assert out[3] == 0.0 and np.isnan(out[4])


def test_plugin_identity_defenses_read_their_config():
    """robust_learning_rate / weak_dp are accepted on the plugin path (FedML
    builds them but hooks neither); a missing config value raises at
    construction, as FedMLDefender.init does through their __init__."""
    from types import SimpleNamespace

    from fedml_amd.server_aggregator import _check_flags

    _check_flags(SimpleNamespace(enable_defense=True, defense_type="robust_learning_rate", robust_threshold=4))
    _check_flags(SimpleNamespace(enable_defense=True, defense_type="weak_dp", stddev=0.1))
    with pytest.raises(AttributeError):
        _check_flags(SimpleNamespace(enable_defense=True, defense_type="robust_learning_rate"))
    with pytest.raises(AttributeError):
        _check_flags(SimpleNamespace(enable_defense=True, defense_type="weak_dp"))
    with pytest.raises(NotImplementedError):
        _check_flags(SimpleNamespace(enable_defense=True, defense_type="foolsgold"))


@pytest.mark.parametrize("dt,full", [
    ("krum", dict(byzantine_client_num=1)),
    ("multikrum", dict(byzantine_client_num=1)),
    ("norm_diff_clipping", dict(norm_bound=0.5)),
    ("cclip", dict(bucket_size=2)),
    ("slsgd", dict(trim_param_b=1, alpha=0.5, option_type=2)),
])
def test_before_aggregation_defenses_read_their_config_at_construction(dt, full):
    """The defenders' constructors read their config values at
    FedMLDefender.init (krum_defense.py:20, norm_diff_clipping_defense.py:17,
    cclip_defense.py:23, slsgd_defense.py:30-34): each missing one raises
    AttributeError when the server aggregator is built, not at the first
    round.  SLSGD checks alpha's bound before reading option_type."""
    from types import SimpleNamespace

    from fedml_amd.server_aggregator import MI355XServerAggregator

    MI355XServerAggregator(torch.nn.Linear(2, 2), SimpleNamespace(enable_defense=True, defense_type=dt, **full))
    for drop in full:
        args = SimpleNamespace(enable_defense=True, defense_type=dt,
                               **{k: v for k, v in full.items() if k != drop})
        with pytest.raises(AttributeError):
            MI355XServerAggregator(torch.nn.Linear(2, 2), args)
    if dt == "slsgd":
        with pytest.raises(ValueError):
            MI355XServerAggregator(torch.nn.Linear(2, 2),
                                   SimpleNamespace(enable_defense=True, defense_type=dt, trim_param_b=1, alpha=2))


def test_robust_learning_rate_host_checks_before_device_work():
    """The reference's behaviour that needs no GPU: threshold 0 hands the list
    to the base function untouched; Σn = 0 raises ZeroDivisionError (at the
    first weight, as `local_sample_number / total_sample_num` does); a bf16
    model is refused by name rather than aggregated another way."""
    raw = [(3, OrderedDict(w=torch.ones(4))), (5, OrderedDict(w=torch.zeros(4)))]
    seen = []
    assert dfn.robust_learning_rate(raw, 0, lambda lst: seen.append(lst) or "base") == "base"
    assert seen == [raw]
    with pytest.raises(ZeroDivisionError):
        dfn.robust_learning_rate([(0, OrderedDict(w=torch.ones(2))), (0, OrderedDict(w=torch.ones(2)))], 1)
    with pytest.raises(NotImplementedError):
        dfn.robust_learning_rate([(1, OrderedDict(w=torch.ones(2, dtype=torch.bfloat16)))], 1)
    d = dfn.RobustLearningRateDefense(type("A", (), {"robust_threshold": 0})())
    assert d.run(raw, lambda lst: "base") == "base" and d.get_malicious_client_idxs() == []


def test_gram_condition_from_distances():
    """dfn.gram_condition recovers the client-mean-centred norms from D alone
    (double centring) and reports max (|c_i|^2 + |c_j|^2) / D_ij: about 1 for
    iid clients, large when one update sits far away, inf for two distinct
    clients at distance 0; 0 below two clients."""
    rng = np.random.default_rng(0)
    X = 0.05 * rng.standard_normal(2000) + 0.01 * rng.standard_normal((30, 2000))

    def D_of(X):
        d = X[:, None, :] - X[None, :, :]
        return (d * d).sum(-1)

    C = X - X.mean(0)
    c2 = (C * C).sum(1)
    D = D_of(X)
    off = ~np.eye(30, dtype=bool)
    want = ((c2[:, None] + c2[None, :])[off] / D[off]).max()
    assert abs(dfn.gram_condition(D) - want) < 1e-9 * want
    assert 0.5 < dfn.gram_condition(D) < 2.0
    X2 = X.copy()
    X2[3] *= 1e3
    assert dfn.gram_condition(D_of(X2)) > 1e3
    X3 = X.copy()
    X3[4] = X3[5]
    assert dfn.gram_condition(D_of(X3)) == float("inf")
    assert dfn.gram_condition(np.zeros((1, 1))) == 0.0
    assert dfn.gram_condition(np.zeros((3, 3))) == 0.0  # all clients identical: nothing to lose


class _OnDevice(torch.Tensor):
    """A host tensor that reports a CUDA device (the placement check reads
    only .is_cuda and .device)."""
    _dev = None

    @property
    def is_cuda(self):
        return True

    @property
    def device(self):
        return self._dev


def _on(t, i):
    t = t.as_subclass(_OnDevice)
    t._dev = torch.device("cuda", i)
    return t


def test_defenses_refuse_a_round_spread_over_gpus():
    """A round whose weight keys sit on several GPUs (a MultiDeviceBucket's
    views) gets a clear NotImplementedError from the gathering defenses
    instead of an out-of-memory error inside the gather."""
    d = OrderedDict([("a.weight", _on(torch.zeros(3), 0)), ("b.weight", _on(torch.zeros(2), 1)),
                     ("bn.running_mean", _on(torch.zeros(2), 2))])
    with pytest.raises(NotImplementedError, match="spread over 2 GPUs"):
        dfn._one_device(d, ["a.weight", "b.weight"], "krum")
    dfn._one_device(d, ["a.weight"], "krum")  # one device: fine
    with pytest.raises(NotImplementedError, match="wise_median"):
        dfn.coordinate_wise_median([(1, d), (1, d)])


def test_median_row_dtype_follows_torch_cat():
    """The median's row dtype is torch.cat's promoted dtype for every mix of
    weight-key dtypes it accepts; the mixes it refuses are the ones whose
    promotion is not exact in fp32 rows (16-bit floats with integers) or has
    no float at all."""
    import itertools

    pool = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.bool]
    for r in range(1, 4):
        for dts in itertools.combinations(pool, r):
            cat = torch.cat([torch.zeros(1, dtype=d) for d in dts]).dtype
            floats = set(dts) & {torch.float32, torch.bfloat16, torch.float16}
            if not floats or (floats <= {torch.bfloat16, torch.float16} and len(floats) == 1 and len(dts) > 1):
                with pytest.raises(NotImplementedError, match="wise_median"):
                    dfn.median_row_dtype(dts)
                continue
            assert dfn.median_row_dtype(dts) == cat, dts


def test_oracle_median_zero_ties_take_the_total_order():
    """The oracle's lower median picks -0.0 / +0.0 by the IEEE total order when
    the rank falls among both zeros, whatever the input order."""
    from oracle import fedavg_oracle as orc

    cols = [([0.0, -0.0, 1.0], 0.0), ([-0.0, 0.0, 1.0], 0.0), ([0.0, -0.0, -1.0], -0.0), ([-1.0, 0.0, -0.0], -0.0),
            ([-0.0, -0.0, 0.0, 0.0], -0.0), ([0.0, 0.0, -0.0, 2.0], 0.0), ([2.0, 1.0, 3.0], 2.0)]
    for vals, want in cols:
        got = orc.lower_median_cols(np.array(vals, dtype=np.float32).reshape(-1, 1))[0]
        assert got == want and np.signbit(got) == np.signbit(want), (vals, got)
