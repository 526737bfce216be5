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

import threading
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch

from . import _native as nat

_STAGE: Dict[torch.device, torch.Tensor] = {}  # pinned uint8 staging per device, grown on demand
_LOCK = threading.Lock()  # one caller at a time uses a staging buffer
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


def _span_to_host(dev, ts, keys, lo, hi, into, out) -> None:
    """One buffer's covered byte span through the pinned staging, then the
    native scatter into the per-key host tensors."""
    stage = _stage(dev, hi - lo)
    base = ts[0].untyped_storage().data_ptr()
    span = torch.empty(0, dtype=torch.uint8, device=dev)
    span.set_(ts[0].untyped_storage(), lo - base, (hi - lo,))
    with torch.cuda.device(dev):
        stage[:hi - lo].copy_(span)  # one DMA, ordered after the producers on the current stream
    dsts, srcs, nbs = [], [], []
    sp = stage.data_ptr()
    for k, t in zip(keys, ts):
        dst = into.get(k) if into is not None else None
        if not (isinstance(dst, torch.Tensor) and not dst.is_cuda and dst.is_contiguous()
                and dst.dtype == t.dtype and tuple(dst.shape) == tuple(t.shape)):
            dst = torch.empty(t.shape, dtype=t.dtype)
        out[k] = dst
        dsts.append(dst.data_ptr())
        srcs.append(sp + (t.data_ptr() - lo))
        nbs.append(t.numel() * t.element_size())
    d = np.asarray(dsts, dtype=np.int64)
    s = np.asarray(srcs, dtype=np.uint64)
    n = np.asarray(nbs, dtype=np.int64)
    nat.check(nat.lib().fedagg_host_gather(d.ctypes.data, s.ctypes.data, n.ctypes.data, int(n.size),
                                           _GATHER_THREADS), "host_gather")


def _one(t: torch.Tensor, dst) -> torch.Tensor:
    if (isinstance(dst, torch.Tensor) and not dst.is_cuda and dst.is_contiguous() and dst.dtype == t.dtype
            and tuple(dst.shape) == tuple(t.shape)):
        dst.copy_(t)
        return dst
    return t.cpu()
