"""The averaged model back to host memory in one DMA per buffer.

FedML sends the aggregated state dict out from the host (the cross-silo
server pickles it for MQTT / S3 / gRPC, and a CPU-resident server model is
filled with ``load_state_dict``, ``server_aggregator.py`` / ``default_aggregator.py``
``set_model_params``).  Done key by key, that is one pageable D2H per key:
320 copies of ResNet-50's 102 MB ran at 5-8 GB/s on MI355X boxes
(``profiles/r05/e/``).  The drop-in's results are views of one flat device
buffer per dtype group (``ClientBucket.reduce_slots`` / ``new_outputs``,
the walked multi-tensor outputs), so :func:`to_host` copies each underlying
buffer's covered byte span ONCE into pinned memory and scatters the keys out
of it with the library's native thread pool (``fedagg_host_gather``).
Tensors that are not such views (or not on a GPU) are copied one by one, as
before; the results are bit-identical to ``t.cpu()`` either way.
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch

from . import _native as nat

_STAGE: Dict[torch.device, torch.Tensor] = {}  # pinned uint8 staging per device, grown on demand
_LOCK = threading.Lock()  # one caller at a time uses a staging buffer
_STREAMS: Dict[torch.device, "torch.cuda.Stream"] = {}  # D2H copy stream per device
_CHUNK = 16 << 20  # bytes per D2H piece: the scatter of a piece overlaps the next pieces' DMA
_GATHER_THREADS = 15
# a buffer whose keys cover less than this share of the span they sit in is
# copied key by key (a few small views of a big buffer)
_MIN_DENSITY = 0.5


def _stage(device: torch.device, nbytes: int) -> torch.Tensor:
    st = _STAGE.get(device)
    if st is None or st.numel() < nbytes:
        st = _STAGE[device] = torch.empty(max(nbytes, 1), dtype=torch.uint8).pin_memory()
    return st


def to_host(state_dict, into: Optional[Dict[str, torch.Tensor]] = None) -> "OrderedDict[str, torch.Tensor]":
    """Host copies of ``state_dict``'s tensors, in its key order.

    into: host tensors to write instead of allocating (e.g. a CPU model's
    ``state_dict()``, as ``load_state_dict`` would): a key whose ``into``
    tensor is contiguous, on the CPU and of the same dtype and shape is
    written in place and returned; any other key gets a fresh tensor (the
    caller converts it, as ``load_state_dict``'s ``copy_`` does).
    Non-tensor values pass through."""
    out: "OrderedDict[str, object]" = OrderedDict((k, None) for k in state_dict)
    groups: Dict[tuple, list] = {}
    for k, t in state_dict.items():
        if not isinstance(t, torch.Tensor):
            out[k] = t
        elif t.is_cuda and t.is_contiguous() and t.numel() > 0:
            groups.setdefault((t.device, t.untyped_storage().data_ptr()), []).append(k)
        else:
            out[k] = t.cpu() if t.is_cuda else t  # (a host tensor is returned as it is, like .cpu())
    for (dev, _), keys in groups.items():
        ts = [state_dict[k] for k in keys]
        lo = min(t.data_ptr() for t in ts)
        hi = max(t.data_ptr() + t.numel() * t.element_size() for t in ts)
        used = sum(t.numel() * t.element_size() for t in ts)
        if len(keys) == 1 or used < _MIN_DENSITY * (hi - lo):
            for k, t in zip(keys, ts):
                out[k] = _one(t, into.get(k) if into is not None else None)
            continue
        with _LOCK:
            _span_to_host(dev, ts, keys, lo, hi, into, out)
    return out


def _copy_stream(dev: torch.device) -> "torch.cuda.Stream":
    st = _STREAMS.get(dev)
    if st is None:
        st = _STREAMS[dev] = torch.cuda.Stream(dev)
    return st


def _span_to_host(dev, ts, keys, lo, hi, into, out) -> None:
    """One buffer's covered byte span through the pinned staging, then the
    native scatter into the per-key host tensors.  The span goes down in
    _CHUNK pieces on a copy stream (after the producers queued on the
    current stream), and the keys that end in a piece are scattered as soon
    as it has landed, while the next pieces are still on the link."""
    n = hi - lo
    chunk = int(os.environ.get("FEDAGG_TO_HOST_CHUNK", _CHUNK)) or n  # tuning override (0: one piece)
    stage = _stage(dev, n)
    base = ts[0].untyped_storage().data_ptr()
    span = torch.empty(0, dtype=torch.uint8, device=dev)
    span.set_(ts[0].untyped_storage(), lo - base, (n,))
    cuts = list(range(0, n, chunk)) + [n]
    events = []
    with torch.cuda.device(dev):
        cs = _copy_stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            for a, b in zip(cuts[:-1], cuts[1:]):
                stage[a:b].copy_(span[a:b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
                events.append(ev)
        # the span's memory may be freed and reused by the caller's stream only after the copies
        span.record_stream(cs)
    per_chunk = [([], [], []) for _ in events]
    sp = stage.data_ptr()
    for k, t in zip(keys, ts):
        dst = into.get(k) if into is not None else None
        if not (isinstance(dst, torch.Tensor) and not dst.is_cuda and dst.is_contiguous()
                and dst.dtype == t.dtype and tuple(dst.shape) == tuple(t.shape)):
            dst = torch.empty(t.shape, dtype=t.dtype)
        out[k] = dst
        nb = t.numel() * t.element_size()
        off = t.data_ptr() - lo
        d, s_, z = per_chunk[(off + nb - 1) // chunk]  # the piece holding the key's last byte
        d.append(dst.data_ptr())
        s_.append(sp + off)
        z.append(nb)
    for ev, (d, s_, z) in zip(events, per_chunk):
        ev.synchronize()
        if not z:
            continue
        da = np.asarray(d, dtype=np.int64)
        sa = np.asarray(s_, dtype=np.uint64)
        za = np.asarray(z, dtype=np.int64)
        nat.check(nat.lib().fedagg_host_gather(da.ctypes.data, sa.ctypes.data, za.ctypes.data, int(za.size),
                                               _GATHER_THREADS), "host_gather")


def _one(t: torch.Tensor, dst) -> torch.Tensor:
    if (isinstance(dst, torch.Tensor) and not dst.is_cuda and dst.is_contiguous() and dst.dtype == t.dtype
            and tuple(dst.shape) == tuple(t.shape)):
        dst.copy_(t)
        return dst
    return t.cpu()
