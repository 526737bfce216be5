"""FAGG wire format: lossless round trips, the row image, and rejection of
malformed or mismatched messages (CPU)."""
from __future__ import annotations

import struct
from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import wire
from fedml_amd.layout import RowLayout

ROUNDTRIP = [c["name"] for c in cases.CASES if not c.get("triple") and not c.get("drop_key")]


@pytest.mark.parametrize("name", ROUNDTRIP)
def test_roundtrip_is_lossless(name):
    spec = next(c for c in cases.CASES if c["name"] == name)
    for n, d in cases.build_inputs(spec):
        msg = wire.encode(d, n)
        n2, d2 = wire.decode(msg)
        assert n2 == n and type(n2) == type(n)
        assert list(d2.keys()) == list(d.keys())
        for k in d:
            assert d2[k].dtype == d[k].dtype and d2[k].shape == d[k].shape, k
            if d[k].numel():
                assert np.array_equal(gu.bits(d2[k]), gu.bits(d[k])), k


def test_payload_is_the_row_image():
    raw = cases.build_inputs(next(c for c in cases.CASES if c["name"] == "mixed_dtypes_k4"))
    n, d = raw[1]
    msg = wire.encode(d, n)
    lay = RowLayout(d)
    _, regions = wire.row_regions(msg, lay)
    for dt, host in regions:
        g = lay.groups[dt]
        assert host.numel() == g.length
        exp = torch.zeros(g.length, dtype=dt)
        for key, off, cnt in zip(g.keys, g.offsets, g.numels):
            exp[off:off + cnt] = d[key].reshape(-1).to(dt)
        assert np.array_equal(gu.bits(host), gu.bits(exp))
    hdr, base = wire.parse_header(msg)
    assert base % 64 == 0 and all(off % 64 == 0 for _, off, _ in hdr["regions"])


def test_rejects_bad_messages():
    d = OrderedDict(a=torch.ones(5), n=torch.tensor(3))
    msg = wire.encode(d, 7)
    with pytest.raises(wire.WireFormatError):
        wire.decode(b"XXXX" + bytes(msg[4:]))
    bad = bytearray(msg)
    struct.pack_into("<H", bad, 4, 99)
    with pytest.raises(wire.WireFormatError):
        wire.decode(bad)
    with pytest.raises(wire.WireFormatError):
        wire.decode(msg[:-10])
    other = RowLayout(OrderedDict(a=torch.ones(6), n=torch.tensor(3)))
    with pytest.raises(wire.WireFormatError):
        wire.row_regions(msg, other)


def test_no_pickle_in_messages():
    d = OrderedDict(w=torch.randn(10))
    msg = wire.encode(d, 1)
    assert bytes(msg[:2]) != b"\x80\x04" and msg[:4] == b"FAGG"  # not a pickle
