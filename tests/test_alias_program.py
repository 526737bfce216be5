"""The drop-in's handling of a dict listed more than once (CPU).

agg_operator.py:36-44 makes client 0's dict the accumulator, so a later entry
that is the same dict reads the running sum; fedml_amd runs such rounds as a
short program of ordinary weighted reductions (fedml_amd.agg_operator.
_run_cells / sequential_sum_inplace).  Here the reductions themselves are
stubbed with the oracle's per-key chains, so the program's cutting and
chaining logic is checked against the reference's fixtures without a GPU (the
same fixtures run through the real kernels in tests/test_gpu_parity.py).
"""
from __future__ import annotations

from collections import OrderedDict

import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import agg_operator as ao
from oracle import fedavg_oracle as orc


def _stub_weighted_reduce(dicts, keys, weights, args):
    return OrderedDict((k, orc.wsum([d[k] for d in dicts], weights)) for k in keys)


def _stub_seq_sum(per_key, keys, K, args):
    if K < 2:
        return
    for k in keys:
        ts = per_key[k][:K]
        res = orc.seqsum(ts)
        orc._set_inplace(ts[0], orc.from_np(res, ts[0].dtype, ts[0].shape))


@pytest.fixture
def stubbed(monkeypatch):
    monkeypatch.setattr(ao, "weighted_reduce", _stub_weighted_reduce)
    monkeypatch.setattr(ao, "_seq_sum_lists", _stub_seq_sum)


@pytest.mark.parametrize("name", [c["name"] for c in cases.ALIAS_CASES])
def test_alias_program_matches_reference(name, stubbed):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    client0, objs = raw[0][1], dict(raw[0][1])
    before = {k: t.clone() for k, t in objs.items()}
    third = gu.snapshot_third(raw)
    res = ao.FedMLAggOperator.agg(cases.Args(spec), raw)
    gu.assert_groups(res, meta, arrays, name)
    gu.assert_third_mutation(third, meta, arrays, name)
    first = res[0] if isinstance(res, tuple) else res
    assert (first is client0) == meta["result_is_client0_dict"]
    for k, t in objs.items():
        assert (not torch.equal(t, before[k])) == (k in meta["client0_tensors_mutated"]), k


def test_no_alias_takes_one_reduction(stubbed, monkeypatch):
    """Without aliasing the round stays ONE weighted reduction (the fast path)."""
    calls = []
    monkeypatch.setattr(ao, "weighted_reduce", lambda *a: calls.append(a) or _stub_weighted_reduce(*a))

    class A:
        federated_optimizer = "FedAvg"

    raw = [(i + 1, OrderedDict(x=torch.full((3,), float(i)))) for i in range(5)]
    ao.FedMLAggOperator.agg(A(), raw)
    assert len(calls) == 1 and len(calls[0][0]) == 5


def test_alias_chain_pieces(stubbed, monkeypatch):
    """[d0, x1, d0, x3, x4, d0]: the chain is cut at each alias and the next
    piece starts from [acc (w=1), acc (w=w_j), ...]."""
    pieces = []
    monkeypatch.setattr(ao, "weighted_reduce", lambda d, k, w, a: pieces.append(list(w)) or
                        _stub_weighted_reduce(d, k, w, a))

    class A:
        federated_optimizer = "FedAvg"

    d0 = OrderedDict(x=torch.ones(2))
    raw = [(1, d0), (2, OrderedDict(x=torch.ones(2))), (3, d0), (4, OrderedDict(x=torch.ones(2))),
           (5, OrderedDict(x=torch.ones(2))), (6, d0)]
    ao.FedMLAggOperator.agg(A(), raw)
    w = [n / 21 for n in range(1, 7)]
    assert pieces == [w[:2], [1.0, w[2], w[3], w[4]], [1.0, w[5]]]


def test_scaffold_cross_role_alias_is_refused(stubbed):
    class A:
        federated_optimizer = "SCAFFOLD"
        client_num_in_total = 4

    d = OrderedDict(x=torch.ones(2))
    c = OrderedDict(x=torch.ones(2))
    with pytest.raises(NotImplementedError):
        ao.FedMLAggOperator.agg(A(), [(1, d, c), (1, OrderedDict(x=torch.ones(2)), d)])


def test_running_sum_detection():
    t = torch.arange(8.0)
    assert ao._reads_running_sum([t, torch.ones(8), t, t.view(8)]) == [2, 3]
    buf = torch.arange(16.0)
    assert ao._reads_running_sum([buf[0:8], buf[8:16]]) == []  # neighbouring rows of one storage
    with pytest.raises(NotImplementedError):
        ao._reads_running_sum([buf[0:8], buf[4:12]])


def test_interleaved_views_that_share_no_element_are_independent():
    """clients holding different columns of one matrix span
    overlapping byte extents but share no element; the reference's in-place
    FedAvg_seq sum into client 0's column handles them, so they are not
    refused.  A view that does share an element still is."""
    m = torch.arange(24.0).reshape(4, 6)
    cols = [m[:, j] for j in range(6)]
    assert ao._reads_running_sum(cols) == []
    assert not ao._shares_elements(m[:, 0], m[:, 1])
    assert ao._shares_elements(m[:, 0], m[0:2, 0])
    with pytest.raises(NotImplementedError):  # rows 1..3 of column 0: three shared elements
        ao._reads_running_sum([m[:, 0], m.view(-1)[6:24:6]])
    every_other = torch.arange(16.0)
    assert ao._reads_running_sum([every_other[0::2], every_other[1::2]]) == []


def test_fedavg_seq_over_column_views_matches_the_reference_loop():
    """The in-place sum of agg_operator.py:58-63 over column views of one
    matrix (restated with torch ops): client 0's column receives the sum, the
    other columns keep their values.  Host dicts go to the GPU, so this runs
    where a GPU is present."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = torch.randn(5, 4)
    ref = m.clone()
    acc = ref[:, 0]
    for j in range(1, 4):
        acc += ref[:, j]
    raw = [(1.0, OrderedDict(w=m[:, j])) for j in range(4)]

    class A:
        federated_optimizer = "FedAvg_seq"

    ao.FedMLAggOperator.agg(A(), raw)
    assert torch.equal(m, ref)
