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


def _with_header(msg, edit):
    """msg with its JSON header edited in place (same header length)."""
    import json

    hdr, base = wire.parse_header(msg)
    edit(hdr)
    hb = json.dumps(hdr, separators=(",", ":")).encode()
    assert len(hb) <= base - 64
    out = bytearray(msg)
    out[64:base] = hb + b" " * (base - 64 - len(hb))
    return out


@pytest.mark.parametrize("edit", [
    lambda h: h["regions"].pop(),                                   # a dtype group missing
    lambda h: h["regions"][0].__setitem__(2, h["regions"][0][2] - 64),  # short region
    lambda h: h["regions"][0].__setitem__(1, 1 << 30),             # past the payload
    lambda h: h["regions"][0].__setitem__(1, -64),                 # negative offset
    lambda h: h["ints"].pop(),                                      # integer key missing
    lambda h: h["ints"][0].__setitem__(3, 1),                      # wrong side-table size
    lambda h: h["ints"][0].__setitem__(2, 1 << 30),                # side table past the payload
    lambda h: h.__setitem__("regions", "x"),                        # not a list of triples
])
def test_rejects_malformed_headers(edit):
    """Headers from the network are checked against the layout and the
    payload length before any ingest: a short regions list used to leave a
    dtype group's row holding the previous round's bytes (zip truncation)."""
    d = OrderedDict(a=torch.ones(5), h=torch.ones(3, dtype=torch.bfloat16), n=torch.tensor(3))
    msg = wire.encode(d, 7)
    bad = _with_header(msg, edit)
    with pytest.raises(wire.WireFormatError):
        wire.decode(bad)
    with pytest.raises(wire.WireFormatError):
        wire.row_regions(bad, RowLayout(d))
    wire.row_regions(msg, RowLayout(d))  # the unedited message passes


def test_rejects_non_json_header():
    msg = bytearray(wire.encode(OrderedDict(a=torch.ones(5)), 1))
    msg[64:68] = b"\xff\xfe{["
    with pytest.raises(wire.WireFormatError):
        wire.decode(msg)
