"""Flat client-update wire format "FAGG" v1.

Today a client update crosses the network as ``pickle.dumps(OrderedDict[str,
Tensor])`` (core/distributed/communication/s3/remote_storage.py:75-81,
:215-264; grpc/grpc_comm_manager.py:84,136).  The server unpickles one tensor
per key and FedML then moves them to the device one by one
(ml_engine_adapter.py:234-254, ~12 GB/s measured).

A FAGG message is the client's ClientBucket row image plus a small header, so
the server ingests it with ONE host->device copy per dtype group and no host
packing (``ClientBucket.put_encoded``).  It is lossless: integer keys travel
both as their fl32 row slot (what the reduction reads) and, exactly, in a side
table (what ``decode`` returns).  No pickle: the header is JSON.

Byte layout (little endian):

    0    4   magic b"FAGG"
    4    2   version (1)
    6    2   reserved
    8    4   header length H (bytes, multiple of 64)
    12   4   reserved
    16   8   payload length P (bytes)
    24  40   reserved (zero)
    64   H   header: UTF-8 JSON, space-padded to 64 B
               {"sample_num", "entries": [[key, shape, dtype]], "promote_ints",
                "signature", "regions": [[dtype, offset, nbytes]],
                "ints": [[key, dtype, offset, nbytes]]}
    64+H P   payload: one region per row dtype group (the exact row image of
             fedml_amd.layout.RowLayout, zero gaps, 64-B aligned), then the
             integer side table (each entry 64-B aligned)

Offsets in the header are relative to the payload start.
"""
from __future__ import annotations

import json
import struct
from collections import OrderedDict
from typing import Tuple

import torch

from .layout import RowLayout, numel

MAGIC = b"FAGG"
VERSION = 1
_PRE = 64
_DTYPES = {str(d).replace("torch.", ""): d for d in (torch.float32, torch.bfloat16, torch.float16, torch.float64,
                                                     torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8,
                                                     torch.bool)}


def _dt_name(d: torch.dtype) -> str:
    return str(d).replace("torch.", "")


def _up64(n: int) -> int:
    return (n + 63) // 64 * 64


class WireFormatError(ValueError):
    pass


def _plan(layout: RowLayout):
    regions, off = [], 0
    for dt, g in layout.groups.items():
        nbytes = g.padded * g.esize
        regions.append([_dt_name(dt), off, nbytes])
        off = _up64(off + nbytes)
    ints = []
    for key, shape, dt in layout.entries:
        if key in layout.int_keys:
            nb = numel(shape) * torch.empty((), dtype=dt).element_size()
            ints.append([key, _dt_name(dt), off, nb])
            off = _up64(off + nb)
    return regions, ints, off


def encode(state_dict, sample_num, promote_ints: bool = True) -> bytearray:
    """One host pass over the update; returns the message bytes."""
    layout = RowLayout(state_dict, promote_ints)
    regions, ints, payload_len = _plan(layout)
    header = {
        "sample_num": sample_num,
        "entries": [[k, list(s), _dt_name(d)] for k, s, d in layout.entries],
        "promote_ints": promote_ints,
        "signature": layout.signature(),
        "regions": regions,
        "ints": ints,
    }
    hb = json.dumps(header, separators=(",", ":")).encode()
    H = _up64(len(hb))
    buf = bytearray(_PRE + H + payload_len)
    struct.pack_into("<4sHHIIQ", buf, 0, MAGIC, VERSION, 0, H, 0, payload_len)
    buf[_PRE:_PRE + len(hb)] = hb
    buf[_PRE + len(hb):_PRE + H] = b" " * (H - len(hb))
    base = _PRE + H
    for (dtn, off, _), (dt, g) in zip(regions, layout.groups.items()):
        region = torch.frombuffer(buf, dtype=dt, count=g.padded, offset=base + off)
        for key, o, n in zip(g.keys, g.offsets, g.numels):
            if n:
                region[o:o + n].copy_(state_dict[key].detach().reshape(-1))  # ints: torch's RNE cast to fp32
    for key, dtn, off, nb in ints:
        t = state_dict[key].detach().reshape(-1).contiguous()
        if nb:
            dst = torch.frombuffer(buf, dtype=_DTYPES[dtn], count=t.numel(), offset=base + off)
            dst.copy_(t)
    return buf


def _parse(buf) -> Tuple[dict, int, int]:
    mv = memoryview(buf)
    if len(mv) < _PRE:
        raise WireFormatError("message shorter than the fixed preamble")
    magic, ver, _, H, _, P = struct.unpack_from("<4sHHIIQ", mv, 0)
    if magic != MAGIC:
        raise WireFormatError(f"bad magic {magic!r}")
    if ver != VERSION:
        raise WireFormatError(f"unsupported version {ver}")
    if len(mv) < _PRE + H + P:
        raise WireFormatError(f"truncated message: {len(mv)} < {_PRE + H + P}")
    try:
        header = json.loads(bytes(mv[_PRE:_PRE + H]).decode())
    except (UnicodeDecodeError, ValueError) as e:
        raise WireFormatError(f"header is not JSON: {e}") from None
    if not isinstance(header, dict):
        raise WireFormatError("header is not a JSON object")
    return header, _PRE + H, P


def parse_header(buf) -> Tuple[dict, int]:
    """(header dict, payload start offset); raises WireFormatError."""
    header, base, _ = _parse(buf)
    return header, base


def _check_regions(header: dict, layout: RowLayout, P: int) -> None:
    """The header's region and side-table lists against the layout and the
    payload length: the message comes from the network, so a short list
    (zip would truncate and leave a group's row stale), a wrong size or an
    extent past the payload is a WireFormatError, never a silent partial
    ingest."""
    try:
        regions = [(str(d), int(o), int(n)) for d, o, n in header["regions"]]
        ints = [(str(k), str(d), int(o), int(n)) for k, d, o, n in header["ints"]]
    except (KeyError, TypeError, ValueError):
        raise WireFormatError("malformed regions / ints lists") from None
    if len(regions) != len(layout.groups):
        raise WireFormatError(f"{len(regions)} regions for {len(layout.groups)} dtype groups")
    for (dtn, off, nbytes), (dt, g) in zip(regions, layout.groups.items()):
        if dtn != _dt_name(dt):
            raise WireFormatError("region order does not match the layout")
        if nbytes != g.padded * g.esize:
            raise WireFormatError(f"region {dtn}: {nbytes} bytes, layout needs {g.padded * g.esize}")
        if off < 0 or off % g.esize or off + nbytes > P:
            raise WireFormatError(f"region {dtn} [{off}, {off + nbytes}) outside the {P}-byte payload")
    want = {k: dt for k, _, dt in layout.entries if k in layout.int_keys}
    if len(ints) != len(want) or {k for k, _, _, _ in ints} != set(want):
        raise WireFormatError("integer side table does not list the layout's integer keys")
    shapes = {k: s for k, s, _ in layout.entries}
    for key, dtn, off, nb in ints:
        if dtn not in _DTYPES or _DTYPES[dtn] != want[key]:
            raise WireFormatError(f"integer key {key!r}: dtype {dtn}")
        if nb != numel(shapes[key]) * torch.empty((), dtype=want[key]).element_size():
            raise WireFormatError(f"integer key {key!r}: {nb} bytes")
        if off < 0 or off + nb > P:
            raise WireFormatError(f"integer key {key!r} outside the payload")


def layout_of(header: dict) -> RowLayout:
    ents = [(k, tuple(s), _DTYPES[d]) for k, s, d in header["entries"]]
    lay = RowLayout(ents, header["promote_ints"])
    if lay.signature() != header["signature"]:
        raise WireFormatError("header signature does not match its entries")
    return lay


def decode(buf) -> Tuple[object, "OrderedDict[str, torch.Tensor]"]:
    """(sample_num, state dict).  Float keys are zero-copy views into buf (keep
    it alive); integer keys come exactly from the side table."""
    header, base, P = _parse(buf)
    lay = layout_of(header)
    _check_regions(header, lay, P)
    regions = {r[0]: r for r in header["regions"]}
    ints = {k: (dtn, off, nb) for k, dtn, off, nb in header["ints"]}
    out = OrderedDict()
    for key, shape, dt in lay.entries:
        if key in ints:
            dtn, off, nb = ints[key]
            n = numel(shape)
            t = torch.frombuffer(buf, dtype=_DTYPES[dtn], count=n, offset=base + off) if n else \
                torch.empty(0, dtype=_DTYPES[dtn])
            out[key] = t.view(shape)
            continue
        g, j = lay.where[key]
        _, roff, _ = regions[_dt_name(g.dtype)]
        n = g.numels[j]
        if n:
            t = torch.frombuffer(buf, dtype=g.dtype, count=n, offset=base + roff + g.offsets[j] * g.esize)
        else:
            t = torch.empty(0, dtype=g.dtype)
        out[key] = t.view(shape)
    return header["sample_num"], out


def row_regions(buf, layout: RowLayout):
    """For ClientBucket.put_encoded: [(dtype, host tensor of the row image)]
    after checking that the message was encoded for exactly this layout."""
    header, base, P = _parse(buf)
    if header.get("signature") != layout.signature():
        raise WireFormatError("update was encoded for a different model layout")
    _check_regions(header, layout, P)
    out = []
    for (dtn, off, nbytes), (dt, g) in zip(header["regions"], layout.groups.items()):
        out.append((dt, torch.frombuffer(buf, dtype=dt, count=g.length, offset=base + off) if g.length else None))
    return header["sample_num"], out
