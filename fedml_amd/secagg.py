"""LightSecAgg server-side field arithmetic on MI355X.

Mirrors, on the same numpy inputs and with identical results:

  aggregate_models_in_finite(weights_finite, prime_number)
      core/mpc/lightsecagg.py:134-148 — per key, w = x_0; w = (w + x_i) mod p
      over clients (numpy int64: wrapping adds, floor modulo).
  model_reconstruction(model_dict, active_clients, aggregate_mask, p, q_bits)
      the per-key loop of LightSecAggAggregator.aggregate_model_reconstruction
      (cross_silo/lightsecagg/lsa_fedml_aggregator.py:139-166): sum the masked
      finite models of the first-round survivors, cancel the decoded
      aggregate mask, mod p, de-quantize (my_q_inv / transform_finite_to_tensor,
      lightsecagg.py:157-182) and scale by 1/K — fused into ONE launch.

The mask itself is decoded from the clients' encoded-mask shares by Lagrange
coded computing (LCC_decoding_with_points, lightsecagg.py); that small
finite-field linear algebra stays with the caller (FedML's own numpy code),
only the model-sized passes run here.
"""
from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Dict, List, Sequence

import numpy as np
import torch

from . import _native as nat
from .bucket import ClientBucket


def _device(device) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise nat.FedAggNativeError("fedml_amd needs a GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _int64_layout(d: "OrderedDict") -> list:
    lay = []
    for k, v in d.items():
        a = np.asarray(v)
        if a.dtype != np.int64:
            raise TypeError(f"key {k!r}: finite-field tensors are int64 (got {a.dtype})")
        lay.append((k, tuple(a.shape), torch.int64))
    return lay


def _fill(bucket: ClientBucket, dicts: Sequence["OrderedDict"]) -> None:
    for i, d in enumerate(dicts):
        # np.ascontiguousarray would turn a 0-d key into shape (1,)
        bucket.put(i, {k: torch.from_numpy(np.array(v, dtype=np.int64, order="C", copy=True)) for k, v in d.items()}, 1)
    bucket.sync_ingest()


def aggregate_models_in_finite(weights_finite: List["OrderedDict"], prime_number: int, device=None
                               ) -> "OrderedDict":
    """lightsecagg.py:134-148 on the GPU; returns a new dict of int64 arrays."""
    p = int(prime_number)
    K = len(weights_finite)
    w_sum = copy.copy(weights_finite[0])  # the reference deep-copies client 0's dict
    layout = _int64_layout(weights_finite[0])
    dev = _device(device)
    with torch.cuda.device(dev):
        bucket = ClientBucket(layout, K, dev, promote_ints=False)
        _fill(bucket, weights_finite)
        g = bucket.groups[torch.int64]
        out = torch.empty(g.padded, dtype=torch.int64, device=dev)
        nat.check(nat.lib().fedagg_sum_mod_i64(g.d_ptrs.data_ptr(), K, g.length, p, out.data_ptr(),
                                               nat.FEDAGG_ALIGNED16, nat.stream_handle()), "sum_mod_i64")
        host = out[:g.length].cpu().numpy()
    for key, off, n, shape in zip(g.keys, g.offsets, g.numels, g.shapes):
        w_sum[key] = host[off:off + n].reshape(shape).copy()
    return w_sum


def model_reconstruction(model_dict: Dict[int, "OrderedDict"], active_clients: Sequence[int],
                         aggregate_mask: np.ndarray, prime_number: int, precision_parameter: int,
                         device=None) -> "OrderedDict":
    """The model-sized part of aggregate_model_reconstruction (:139-166):
    returns model_dict[active_clients[0]] with every key rebound to its float32
    average, as the reference does."""
    p = int(prime_number)
    q = int(precision_parameter)
    K = len(active_clients)
    dicts = [model_dict[c] for c in active_clients]
    averaged_params = dicts[0]
    layout = _int64_layout(averaged_params)
    mask = np.asarray(aggregate_mask).reshape(-1)
    w = 1 / K  # :163, a Python float, rounded to fp32 by torch's mul
    dev = _device(device)
    with torch.cuda.device(dev):
        bucket = ClientBucket(layout, K, dev, promote_ints=False)
        _fill(bucket, dicts)
        g = bucket.groups[torch.int64]
        # the decoded mask, cut per key exactly as :147-151 does, in the row layout
        mrow = np.zeros(g.padded, dtype=np.int64)
        pos = 0
        for off, n in zip(g.offsets, g.numels):
            mrow[off:off + n] = mask[pos:pos + n]
            pos += n
        d_mask = torch.from_numpy(mrow).to(dev)
        out = torch.empty(g.padded, dtype=torch.float32, device=dev)
        nat.check(nat.lib().fedagg_lsa_reconstruct_f32(g.d_ptrs.data_ptr(), K, g.length, d_mask.data_ptr(), p, q,
                                                       float(np.float32(w)), out.data_ptr(), nat.FEDAGG_ALIGNED16,
                                                       nat.stream_handle()), "lsa_reconstruct_f32")
        host = out[:g.length].cpu()
    for key, off, n, shape in zip(g.keys, g.offsets, g.numels, g.shapes):
        # a 0-d key comes back from my_q_inv as a numpy scalar, which
        # transform_finite_to_tensor wraps as torch.Tensor([x]): shape (1,)
        averaged_params[key] = host[off:off + n].clone().reshape(shape if len(shape) else (1,))
    return averaged_params
