"""The native dict walker's host-side entry points (CPU; csrc/walker.cpp).

same_values decides whether a round's dicts are still the bucket views the
cross-silo ingest bound them to (agg_operator._reduce_resident); walk_host of
one dict gives the cross-silo ingest its pointer tables (put_from_table,
col=0)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

from fedml_amd import _native as nat
from fedml_amd import agg_operator as ao


@pytest.fixture(scope="module")
def w():
    m = ao._walker()
    if m is None:
        pytest.skip("walker not built")
    return m


def test_same_values_is_object_identity(w):
    a, b = torch.ones(3), torch.zeros(2)
    view = OrderedDict(x=a, y=b)
    d = OrderedDict(x=a, y=b)
    assert w.same_values([d], [view], ["x", "y"]) is True
    assert w.same_values([d, d], [view, view], ["x"]) is True
    d2 = OrderedDict(x=a.clone(), y=b)  # equal values, another object: not the view
    assert w.same_values([d2], [view], ["x", "y"]) is False
    assert w.same_values([OrderedDict(x=a)], [view], ["x", "y"]) is False  # a missing key
    assert w.same_values([d], [view, view], ["x"]) is False  # list lengths differ


def test_same_values_declines_overriding_dicts(w):
    class Lying(dict):
        def __getitem__(self, k):
            return torch.full((3,), 7.0)

    a = torch.ones(3)
    assert w.same_values([Lying(x=a)], [OrderedDict(x=a)], ["x"]) is False


def test_walk_host_of_one_dict_is_a_one_column_table(w):
    d = OrderedDict(a=torch.arange(5, dtype=torch.float32), n=torch.tensor(3), b=torch.ones(2, 3),
                    h=torch.ones(4, dtype=torch.bfloat16))
    codes, numels, tables = w.walk_host([d], list(d))
    t = {c: np.frombuffer(v, dtype=np.int64).reshape(-1, 1) for c, v in tables.items()}
    assert list(numels) == [5, 1, 6, 4]
    assert t[nat.DT_F32][:, 0].tolist() == [d["a"].data_ptr(), d["b"].data_ptr()]
    assert t[nat.DT_I64][:, 0].tolist() == [d["n"].data_ptr()]
    assert t[nat.DT_BF16][:, 0].tolist() == [d["h"].data_ptr()]
    assert w.walk_host([OrderedDict(a=torch.ones(4)[::2])], ["a"]) is None  # non-contiguous: declined
