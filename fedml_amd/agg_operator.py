"""Drop-in replacement of FedML's aggregation operator, computed on MI355X.

Mirrors python/fedml/ml/aggregator/agg_operator.py (same names, argument
meaning, return values, aliasing and exceptions):

  FedMLAggOperator.agg(args, raw_grad_list)            agg_operator.py:8-30
  model_aggregator(args, raw_grad_list, training_num)   :223-234
  torch_aggregator(args, raw_grad_list, training_num)   :33-134

Every reduction runs in libfedagg.so (include/fedagg.h); there is no CPU
arithmetic and no CPU fallback.  Where the reference's tensors already live on
the GPU (server `using_gpu`, ml_engine_adapter.py:234-254) the kernels read
them in place through pointer tables — all fp32 keys in ONE launch; host
tensors are packed per client into pinned staging rows, copied to HBM, reduced
with one launch per dtype, and copied back, so the result lives where the
inputs did, as in the reference.

Options read from ``args`` (all optional, duck-typed like FedML's Arguments):
  fedagg_device             torch device for host inputs (default: current GPU)
  fedagg_low_precision_acc  "reference" (default: bf16/f16 rounded after every
                            op, bit-exact with torch's CPU chain) or "fp32"
                            (accumulate in fp32, round once)
"""
from __future__ import annotations

import weakref
from collections import OrderedDict
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import _native as nat
from . import kernels as kn
from . import multidev
from .bucket import ClientBucket

_ACC_NAME = {kn.ACC_REFERENCE: "reference", kn.ACC_FP32: "fp32"}

# torch promotes `int_tensor * python_float` to the default dtype float32.
_INT_TO_I64 = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
_FLOAT = (torch.float32, torch.bfloat16, torch.float16, torch.float64)
_SUM_DTYPES = (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32)


class FedMLAggOperator:
    """Same interface as fedml.ml.aggregator.agg_operator.FedMLAggOperator."""

    @staticmethod
    def agg(args, raw_grad_list: List[Tuple[float, "OrderedDict"]]) -> "OrderedDict":
        # agg_operator.py:11-28 — Σ n_i with the same tuple unpacking (and so the
        # same ValueError on a wrong arity).
        training_num = 0
        if args.federated_optimizer in ("SCAFFOLD", "Mime"):
            for i in range(len(raw_grad_list)):
                local_sample_num, _, _ = raw_grad_list[i]
                training_num += local_sample_num
        else:
            for i in range(len(raw_grad_list)):
                local_sample_num, local_model_params = raw_grad_list[i]
                training_num += local_sample_num
        return model_aggregator(args, raw_grad_list, training_num)


def model_aggregator(args, raw_grad_list, training_num):
    """agg_operator.py:223-234.  Only the torch engine is on the MI355X path."""
    engine = getattr(args, "ml_engine", None)
    if engine in ("tf", "jax", "mxnet"):
        raise NotImplementedError(f"fedml_amd aggregates torch state dicts; ml_engine={engine!r} is not supported")
    return torch_aggregator(args, raw_grad_list, training_num)


def _acc_mode(args) -> int:
    mode = getattr(args, "fedagg_low_precision_acc", "reference")
    if mode == "reference":
        return kn.ACC_REFERENCE
    if mode == "fp32":
        return kn.ACC_FP32
    raise ValueError(f"fedagg_low_precision_acc must be 'reference' or 'fp32', got {mode!r}")


def _host_device(args) -> torch.device:
    dev = getattr(args, "fedagg_device", None)
    if dev is not None:
        return torch.device(dev)
    if not torch.cuda.is_available():
        raise nat.FedAggNativeError("fedml_amd needs a GPU: host inputs are reduced on the device")
    return torch.device("cuda", torch.cuda.current_device())


def _gather(dicts: Sequence["OrderedDict"], keys: Sequence[str]) -> Dict[str, List[torch.Tensor]]:
    """Per-key client tensors; KeyError for a missing key, as the reference's
    `local_model_params[k]` raises."""
    out = {}
    for k in keys:
        ts = [d[k] for d in dicts]
        t0 = ts[0]
        s0, d0, g0 = t0.shape, t0.dtype, t0.get_device()
        for t in ts:  # cheap attribute checks first (40,960 tensors at config 3)
            if t.shape != s0 or t.dtype is not d0 or t.get_device() != g0:
                _raise_mismatch(k, t0, t)
        if d0 not in _FLOAT and d0 not in _INT_TO_I64:
            raise TypeError(f"key {k!r}: unsupported dtype {d0}")
        out[k] = ts
    return out


def _raise_mismatch(k: str, t0: torch.Tensor, t: torch.Tensor) -> None:
    if t.shape != t0.shape:
        raise RuntimeError(f"key {k!r}: client tensor shapes differ ({tuple(t.shape)} vs {tuple(t0.shape)})")
    if t.dtype != t0.dtype:
        raise TypeError(f"key {k!r}: client tensor dtypes differ ({t.dtype} vs {t0.dtype})")
    raise RuntimeError(f"key {k!r}: client tensors on different devices ({t.device} vs {t0.device})")


# ---------------------------------------------------------------------------
# Reduction engine


_BUCKETS: "OrderedDict[tuple, ClientBucket]" = OrderedDict()
_BUCKET_CACHE_SIZE = 2


def _cached_bucket(layout, K: int, device: torch.device, acc: str, promote_ints: bool = True) -> ClientBucket:
    """Host-input rounds reuse their HBM rows and pinned staging: a server
    aggregates the same model shape every round (LRU of 2 layouts)."""
    key = (tuple((k, s, str(d)) for k, s, d in layout), K, str(device), acc) + (() if promote_ints else ("exact",))
    b = _BUCKETS.pop(key, None)
    if b is None:
        b = ClientBucket(layout, K, device, low_precision_acc=acc, promote_ints=promote_ints)
        while len(_BUCKETS) >= _BUCKET_CACHE_SIZE:
            _BUCKETS.popitem(last=False)
    _BUCKETS[key] = b
    return b


def _walker():
    """The native dict walker (csrc/walker.cpp), or None if it is not built;
    without it the Python walk below does the same job, slower."""
    global _WALKER
    if _WALKER is False:
        try:
            import importlib.util
            import os

            from . import build as fbuild

            spec = importlib.util.spec_from_file_location("_fedagg_walker", fbuild.WALKER_OUT)
            if spec is None or not os.path.exists(fbuild.WALKER_OUT):
                raise ImportError(fbuild.WALKER_OUT)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            _WALKER = mod
        except (ImportError, OSError):
            _WALKER = None
    return _WALKER


_WALKER = False
_CODE_DT = {nat.DT_F32: torch.float32, nat.DT_BF16: torch.bfloat16, nat.DT_F16: torch.float16,
            nat.DT_I64: torch.int64}


_PLANS: "OrderedDict[tuple, kn.MultiPlan]" = OrderedDict()


def _multi_plan(numels: Sequence[int], code: int, acc_mode: int) -> kn.MultiPlan:
    """Segment tables of the multi-tensor launch, cached per key-size list: a
    server aggregates the same model every round."""
    key = (tuple(numels), code, acc_mode)
    plan = _PLANS.pop(key, None)
    if plan is None:
        plan = kn.MultiPlan(numels, _CODE_DT[code], acc_mode)
        while len(_PLANS) >= 32:
            _PLANS.popitem(last=False)
    _PLANS[key] = plan
    return plan


# Pipelined device path: keys are walked largest first in chunks, and each
# chunk is launched as soon as it is walked, so the GPU reduces the bulk of the
# bytes while the host is still walking the many small keys.
# first chunks small so the GPU starts early, then the rest in 96s.  Config 3
# (tools/devdict_bench.py --chunks): 4,12,48 -> 2.52 ms per agg(), 8,24,64 ->
# 2.55, 16,32,64 -> 2.61, 32,64 -> 2.61, 2,6,24,64 -> 2.57.
_CHUNK_KEYS = (4, 12, 48)
_TAIL_CHUNK = 96  # keys per chunk after _CHUNK_KEYS
# Chunks from this index on hold only small keys (ResNet-50: 87K of 25.6M
# elements over 256 keys).  Their launches are bound by the 128-deep client
# chain per element, not by bytes (26-52 us each at config 3), so they go to a
# side stream and run beside the big HBM-bound launches instead of after them.
_SIDE_FROM_CHUNK = len(_CHUNK_KEYS)
_SIDE: Dict[torch.device, "torch.cuda.Stream"] = {}
# The weights go up with the first chunk's pointer table (one H2D, not two).
_WEIGHTS_IN_TABLE = True


def _side_stream(device: torch.device) -> "torch.cuda.Stream":
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device)
    return s


def _chunks(order: Sequence[int]):
    lo = 0
    for n in _CHUNK_KEYS:
        if lo >= len(order):
            return
        yield order[lo:lo + n]
        lo += n
    while lo < len(order):
        yield order[lo:lo + _TAIL_CHUNK]
        lo += _TAIL_CHUNK


def _device_chunks(groups):
    """(chunk index within its device, key indices) over every device's keys:
    each device's own chunk schedule, the devices interleaved, so every GPU
    gets its largest keys early (a multi-device bucket's views put a round on
    several GPUs, fedml_amd.multidev)."""
    its = [enumerate(_chunks(order)) for _, order in groups]
    while its:
        nxt = []
        for it in its:
            got = next(it, None)
            if got is not None:
                yield got
                nxt.append(it)
        its = nxt


def _reduce_device_walked(w, dicts, keys, weights, acc_mode) -> "OrderedDict[str, torch.Tensor] | None":
    """Every key a contiguous, 16-byte aligned device tensor of one device
    (what the native walker verifies): one multi-tensor launch per dtype and
    chunk with the walker's pointer tables and natively allocated outputs, no
    per-tensor Python work.  None if the walker declines any chunk (the caller
    then runs the general path, which raises the reference's errors; launches
    already made for earlier chunks only wrote outputs nobody sees)."""
    groups = w.group_by_device(dicts[0], keys) if hasattr(w, "group_by_device") else None
    if groups is None:
        order = w.order_by_size(dicts[0], keys)
        if order is None:
            return None
        groups = [(None, order)]
    K = len(dicts)
    results: Dict[str, torch.Tensor] = {}
    keep = []  # device tables of the launches, alive until enqueued
    w32 = {}  # device -> the weights there (the walker checks one device per chunk, not across chunks)
    start = {}  # device -> event on the caller's stream before this call's first kernel there
    joins = []  # (caller's stream, side stream) pairs to rejoin before returning
    try:
        for ci, idx in _device_chunks(groups):
            ck = [keys[i] for i in idx]
            walked = w.walk(dicts, ck, True)
            if walked is None:
                return None
            dev_idx, codes, numels, tables, outs, out_tables = walked
            device = torch.device("cuda", dev_idx)
            with torch.cuda.device(device):
                cur = torch.cuda.current_stream(device)

                def mark_start(device=device, cur=cur):
                    # what the caller's stream queued before this call (the
                    # inputs' producers, earlier users of the outputs' memory)
                    # and the weights' upload, but none of this call's kernels
                    if device not in start:
                        start[device] = torch.cuda.Event()
                        start[device].record(cur)

                side = ci >= _SIDE_FROM_CHUNK and bool(tables)
                if device not in w32 and (side or not _WEIGHTS_IN_TABLE):
                    w32[device] = kn.upload_f32(weights, device)
                    mark_start()
                st = cur
                if side:
                    st = _side_stream(device)
                    # the side launches run beside this call's big launches
                    st.wait_event(start[device])
                    if (cur, st) not in joins:
                        joins.append((cur, st))
                with torch.cuda.stream(st):
                    for code, tab in tables.items():
                        ns = [n for n, c in zip(numels, codes) if c == code]
                        plan = _multi_plan(ns, code, acc_mode)
                        if device not in w32:  # the weights ride in the first table's H2D
                            ret = plan.launch(tab, out_tables[code], None, K, device, weights=weights,
                                              on_uploaded=mark_start)
                            w32[device] = ret[-1]
                        else:
                            ret = plan.launch(tab, out_tables[code], w32[device], K, device)
                        keep.append(ret)
            results.update(zip(ck, outs))
    finally:
        # the caller's stream waits for the side launches, also when a later
        # chunk is declined (their outputs are then freed into its pool)
        for cur, st in joins:
            cur.wait_stream(st)
    return OrderedDict((k, results[k]) for k in keys)


# Buckets whose slot views callers hold as client dicts (the cross-silo
# mirror rebinds every arriving update to its slot's views): a round over
# exactly such dicts reduces the bucket's rows with one launch per dtype
# group, with no walk over K x keys tensors.
_RESIDENT: "weakref.WeakSet" = weakref.WeakSet()


def register_resident(bucket) -> None:
    _RESIDENT.add(bucket)


def _reduce_resident(w, dicts, keys, weights, acc_mode) -> "OrderedDict[str, torch.Tensor] | None":
    """The round's dicts are ALL dicts a registered bucket (a ClientBucket,
    or a MultiDeviceBucket: each device its keys) bound to its slots
    (identity), with the bucket's keys in its order, and every value is still
    that slot's view (the native same_values check): reduce those rows in the
    list's order.  The same kernels and client order as the walked
    path, so the same bits.  Else None."""
    if not _RESIDENT or not hasattr(w, "same_values"):
        return None
    for b in list(_RESIDENT):
        if not b._slot_dicts or b.acc_mode != acc_mode:
            continue
        slots = []
        for d in dicts:
            s = b._slot_of.get(id(d))
            if s is None or b._slot_dicts[s][0] is not d:
                break
            slots.append(s)
        else:
            if list(keys) != b.entry_keys:
                return None
            if not w.same_values(list(dicts), [b._slot_dicts[s][1] for s in slots], list(keys)):
                return None
            return b.reduce_slots(slots, weights)
    return None


_HOST_ROUND_MAX_BYTES = 32 << 20  # host rounds up to this size: one native call, host to host
_HOST_ROUND_FN: "int | None" = None


def _reduce_host_round(w, dicts, keys, weights) -> "OrderedDict[str, torch.Tensor] | None":
    """Small host rounds of fp32 / int64 keys (configs 1 and 2): the whole
    round in ONE native call, fedagg_host_round_f32 (pack into pinned memory,
    reduce on the GPU, results into new fp32 host tensors; no torch copies,
    events or stream bookkeeping around it).  None when the walker declines
    (other dtypes, a non-contiguous or device tensor, K > 256, a bigger round)."""
    global _HOST_ROUND_FN
    if _HOST_ROUND_FN is None:
        import ctypes

        _HOST_ROUND_FN = ctypes.cast(nat.lib().fedagg_host_round_f32, ctypes.c_void_p).value
    # stream 0: the library's own non-blocking stream (host in, host out)
    got = w.host_round(dicts, keys, weights, _HOST_ROUND_FN, 0, _HOST_ROUND_MAX_BYTES)
    if got is None:
        return None
    rc, outs = got
    nat.check(rc, "fedagg_host_round_f32")
    return OrderedDict(zip(keys, outs))


_DEVICE_ROUND_FN: "int | None" = None
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _reduce_device_round(w, dicts, keys, weights) -> "OrderedDict[str, torch.Tensor] | None":
    """Small device rounds of fp32 / int64 keys (config 1 on a `using_gpu`
    server): ONE native call validates the K dicts, allocates the outputs and
    launches fedagg_device_round_f32 with every pointer and weight in the
    kernel arguments, on the device's current stream; no uploads, plans or
    stream lookups in Python.  None when the walker declines (more than 16
    keys or 128 client tensors, other dtypes, unaligned or non-contiguous
    tensors, several devices)."""
    global _DEVICE_ROUND_FN
    if _RAW_STREAM is None or not hasattr(w, "device_round"):
        return None
    if _DEVICE_ROUND_FN is None:
        import ctypes

        _DEVICE_ROUND_FN = ctypes.cast(nat.lib().fedagg_device_round_f32, ctypes.c_void_p).value
    got = w.device_round(dicts, keys, weights, _DEVICE_ROUND_FN, _RAW_STREAM)
    if got is None:
        return None
    rc, outs = got
    nat.check(rc, "fedagg_device_round_f32")
    return OrderedDict(zip(keys, outs))


_BATCH_MAX_BYTES = 256 << 20  # host rounds up to this size stage every client in one pack + one H2D
_ROW_ESZ = {nat.DT_F32: 4, nat.DT_BF16: 2, nat.DT_F16: 2, nat.DT_F64: 8, nat.DT_I64: 8}


def _reduce_host_batched(w, dicts, keys, weights, args, acc_mode) -> "OrderedDict[str, torch.Tensor] | None":
    """Host rounds whose every key is a contiguous CPU tensor of a row dtype:
    the walker's host pointer tables drive the staging, with no per-key
    Python work.  Up to 256 MB per round: ONE native pack of all clients per
    dtype into pinned staging and ONE H2D; larger rounds one pack + one H2D
    per client through the staging ring, so packing client i+1 overlaps
    client i's DMA.  Then one launch per dtype and one D2H.  None when the
    walk declines (the general path then raises the reference's errors)."""
    walked = w.walk_host(dicts, keys)
    if walked is None:
        return None
    codes, numels, tables = walked
    K = len(dicts)
    d0 = dicts[0]
    device = _host_device(args)
    layout = [(k, tuple(d0[k].shape), d0[k].dtype) for k in keys]
    devices = _round_devices(args, layout, K, device, acc_mode)
    if len(devices) > 1:
        return _reduce_host_multi(layout, devices, tables, numels, codes, dicts, weights, acc_mode)
    device = devices[0]  # args.fedagg_devices may name the one device
    with torch.cuda.device(device):
        bucket = _cached_bucket(layout, K, device, _ACC_NAME[acc_mode])
        if K * sum(n * _ROW_ESZ[c] for n, c in zip(numels, codes)) <= _BATCH_MAX_BYTES:
            bucket.put_batch(tables, dicts, [1] * K)
        else:  # large round: per client, packing the next while the last one's DMA runs
            t2d = {c: np.frombuffer(t, dtype=np.int64).reshape(-1, K) for c, t in tables.items()}
            for i in range(K):
                bucket.put_from_table(i, t2d, dicts[i], 1)
        return bucket.reduce_to_host(weights)  # reduce, D2H and host scatter overlapped


_MULTI: "OrderedDict[tuple, multidev.MultiDeviceBucket]" = OrderedDict()


def _round_devices(args, layout, K: int, device: torch.device, acc_mode) -> list:
    """Placement of a host round, decided once per (layout, K, accumulation):
    a bucket already resident for it keeps its devices.  Asking the free HBM
    again would not count that bucket's own rows as free, so a round that fit
    one GPU in round 1 could flip to several GPUs in round 2 and hold its rows
    twice (the cached one-device bucket plus the new shards)."""
    listed = multidev.parse_devices(getattr(args, "fedagg_devices", None))
    lk = tuple((k, s, str(d)) for k, s, d in layout)
    if not listed:
        if (lk, K, str(device), _ACC_NAME[acc_mode]) in _BUCKETS:
            return [device]
        for key in _MULTI:
            if key[0] == lk and key[1] == K and key[3] == acc_mode:
                return [torch.device(d) for d in key[2]]
    elif len(listed) == 1:
        # one device named explicitly: honour it, and drop a multi-device
        # bucket of this layout so its rows do not stay resident beside it
        for key in [k for k in _MULTI if k[0] == lk]:
            del _MULTI[key]
    devices = multidev.devices_for_round(args, layout, K, device)
    if len(devices) > 1:
        # the round goes multi-device: a one-device bucket of the same layout
        # (another K or accumulation) must not stay resident beside it
        lk = tuple((k, s, str(d)) for k, s, d in layout)
        for key in [k for k in _BUCKETS if k[0] == lk]:
            del _BUCKETS[key]
    return devices


def _multi_bucket(layout, K: int, devices, acc_mode) -> "multidev.MultiDeviceBucket":
    """The cached MultiDeviceBucket of this (layout, K, devices, accumulation)."""
    key = (tuple((k, s, str(d)) for k, s, d in layout), K, tuple(str(d) for d in devices), acc_mode)
    b = _MULTI.pop(key, None)
    if b is None:
        _MULTI.clear()  # one multi-device round resident at a time: they are the big ones
        b = multidev.MultiDeviceBucket(layout, K, devices, low_precision_acc=_ACC_NAME[acc_mode])
    _MULTI[key] = b
    return b


def _reduce_host_multi(layout, devices, tables, numels, codes, dicts, weights, acc_mode
                       ) -> "OrderedDict[str, torch.Tensor]":
    """A host round over several GPUs of this process (multidev): whole keys
    per device, each client's keys packed and sent over each device's own
    PCIe link, every device reducing its keys in the reference order (no
    exchange, bit-exact), results scattered back into per-key host tensors.
    The bucket is cached per (layout, K, devices) like the one-device one."""
    K = len(dicts)
    b = _multi_bucket(layout, K, devices, acc_mode)
    t2d = {c: np.frombuffer(t, dtype=np.int64).reshape(-1, K) for c, t in tables.items()}
    per_shard = b.split_tables(t2d)
    if K * sum(n * _ROW_ESZ[c] for n, c in zip(numels, codes)) <= _BATCH_MAX_BYTES:
        b.put_batch(per_shard, dicts, [1] * K)
    else:
        for i in range(K):
            b.put_from_tables(i, per_shard, dicts[i], 1)
    return b.reduce_to_host(weights)


def _multi_requested(args) -> bool:
    return len(multidev.parse_devices(getattr(args, "fedagg_devices", None))) > 1


def weighted_reduce(dicts: Sequence["OrderedDict"], keys: Sequence[str], weights: Sequence[float], args
                    ) -> "OrderedDict[str, torch.Tensor]":
    """avg[k] = Σ_i fl(p_i[k] · w_i) in client order for every key (the FedAvg
    inner loops, agg_operator.py:36-44), on the GPU.  Returns results on the
    inputs' device."""
    acc_mode = _acc_mode(args)
    w = _walker()
    if w is not None and keys:
        dicts, keys = list(dicts), list(keys)
        t0 = dicts[0].get(keys[0]) if isinstance(dicts[0], dict) else None
        if isinstance(t0, torch.Tensor) and not t0.is_cuda and getattr(args, "fedagg_device", None) is None \
                and torch.cuda.is_available() and not multidev.parse_devices(getattr(args, "fedagg_devices", None)):
            res = _reduce_host_round(w, dicts, keys, weights)
            if res is not None:
                return res
        if isinstance(t0, torch.Tensor) and t0.is_cuda:
            res = _reduce_resident(w, dicts, keys, weights, acc_mode)
            if res is not None:
                return res
            if len(keys) <= 16 and len(keys) * len(dicts) <= 128:
                res = _reduce_device_round(w, dicts, keys, weights)
                if res is not None:
                    return res
        res = _reduce_device_walked(w, dicts, keys, weights, acc_mode)
        if res is not None:
            return res
        res = _reduce_host_batched(w, dicts, keys, weights, args, acc_mode)
        if res is not None:
            return res
    per_key = _gather(dicts, keys)
    K = len(dicts)
    results: Dict[str, torch.Tensor] = {}
    host_keys = [k for k in keys if not per_key[k][0].is_cuda]
    dev_keys = [k for k in keys if per_key[k][0].is_cuda]

    # ---- host-resident inputs: pinned staging -> HBM rows, one launch per dtype --
    if host_keys:
        device = _host_device(args)
        layout = [(k, tuple(per_key[k][0].shape), per_key[k][0].dtype) for k in host_keys]
        devices = _round_devices(args, layout, K, device, acc_mode)
        if len(devices) > 1:  # the round spreads over GPUs (fedml_amd.multidev), as on the walked path
            bucket = _multi_bucket(layout, K, devices, acc_mode)
            for i in range(K):
                bucket.put(i, {k: per_key[k][i] for k in host_keys}, 1)
            results.update(bucket.reduce_to_host(weights))
        else:
            device = devices[0]
            with torch.cuda.device(device):
                bucket = _cached_bucket(layout, K, device, _ACC_NAME[acc_mode])
                for i in range(K):
                    bucket.put(i, {k: per_key[k][i] for k in host_keys}, 1)
                results.update(bucket.reduce_to_host(weights))

    # ---- device-resident inputs: read in place --------------------------------
    if dev_keys:
        by_dev: Dict[torch.device, List[str]] = OrderedDict()
        for k in dev_keys:
            by_dev.setdefault(per_key[k][0].device, []).append(k)
        for device, dkeys in by_dev.items():
            with torch.cuda.device(device):
                w32 = kn.upload_f32(weights, device)
                w64 = None
                # one multi-tensor launch per dtype for aligned keys; the rest key by key
                multi: Dict[torch.dtype, Tuple[List[str], List[int], List[int]]] = OrderedDict()
                for k in dkeys:
                    ts = [t if t.is_contiguous() else t.contiguous() for t in per_key[k]]
                    dt = ts[0].dtype
                    if dt in _INT_TO_I64 and dt != torch.int64:
                        ts = [t.to(torch.int64) for t in ts]
                        dt = torch.int64
                    out = torch.empty(ts[0].shape, dtype=torch.float32 if dt == torch.int64 else dt,
                                      device=device)
                    results[k] = out
                    n = out.numel()
                    if n == 0:
                        continue
                    ptrs = [t.data_ptr() for t in ts]
                    if dt in kn.MULTI_DTYPES and kn.aligned16(ptrs) and (out.data_ptr() & 15) == 0:
                        mk, ms, mo = multi.setdefault(dt, ([], [], []))
                        mk.append(k)
                        ms.extend(ptrs)
                        mo.append(out.data_ptr())
                        per_key[k] = ts  # keep any contiguous copies alive
                        continue
                    if dt == torch.float64 and w64 is None:
                        w64 = kn.upload_f64(weights, device)
                    kn.wsum_ptrs(dt, kn.upload_i64(ptrs, device), w64 if dt == torch.float64 else w32, K, n, out,
                                 kn.aligned16(ptrs), acc_mode)
                for dt, (mk, ms, mo) in multi.items():
                    plan = kn.MultiPlan([results[k].numel() for k in mk], dt, acc_mode)
                    plan.launch(ms, mo, w32, K, device)

    return OrderedDict((k, results[k]) for k in keys)


_MULDIV_INT_OK = (torch.int64, torch.bool)


def muldiv_reduce(dicts: Sequence["OrderedDict"], keys: Sequence[str], pairs: Sequence, args
                  ) -> "OrderedDict[str, torch.Tensor]":
    """avg[k] = Σ_i fl(fl(p_i[k]·n_i) / N) in client order for every key, with
    pairs[i] = (n_i, N): the MPI simulation's term order
    (simulation/mpi/fedavg/FedAVGAggregator.py:99-116).  Host keys are staged
    into exact rows (integer keys as int64: `int64 * int` multiplies in int64
    first), device keys are read in place; one fedagg_wsum_muldiv launch per
    dtype group or device key.  Results live where the inputs did."""
    per_key = _gather(dicts, keys)
    K = len(dicts)
    for k in keys:
        dt = per_key[k][0].dtype
        if dt in _INT_TO_I64 and dt not in _MULDIV_INT_OK:
            raise NotImplementedError(f"key {k!r}: {dt} * int wraps at {dt}'s width in torch; "
                                      "fedml_amd's MPI-order path takes int64 / bool integer keys")
    results: Dict[str, torch.Tensor] = {}
    keep = []
    host_keys = [k for k in keys if not per_key[k][0].is_cuda]
    if host_keys:
        device = _host_device(args)
        with torch.cuda.device(device):
            layout = [(k, tuple(per_key[k][0].shape), per_key[k][0].dtype) for k in host_keys]
            bucket = _cached_bucket(layout, K, device, "reference", promote_ints=False)  # exact int64 rows
            for i in range(K):
                bucket.put(i, {k: per_key[k][i] for k in host_keys}, 1)
            bucket.sync_ingest()
            outs = {}
            for dt, g in bucket.groups.items():
                odt = torch.float32 if dt == torch.int64 else dt
                outs[dt] = torch.empty(max(g.length, 1), dtype=odt, device=device)
                if g.length:
                    keep.append(kn.muldiv_ptrs(dt, g.d_ptrs, pairs, K, g.length, outs[dt], True))
            host = {dt: o.cpu() for dt, o in outs.items()}
            for k in host_keys:
                g, j = bucket.where[k]
                results[k] = host[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].view(g.shapes[j]).clone()
    for k in keys:
        if k in results:
            continue
        ts = [t if t.is_contiguous() else t.contiguous() for t in per_key[k]]
        if ts[0].dtype == torch.bool:
            ts = [t.to(torch.int64) for t in ts]
        dt = ts[0].dtype
        device = ts[0].device
        with torch.cuda.device(device):
            out = torch.empty(ts[0].shape, dtype=torch.float32 if dt == torch.int64 else dt, device=device)
            if out.numel():
                ptrs = [t.data_ptr() for t in ts]
                keep.append((ts, kn.muldiv_ptrs(dt, kn.upload_i64(ptrs, device), pairs, K, out.numel(), out,
                                                kn.aligned16(ptrs))))
        results[k] = out
    del keep  # stream-ordered: the caching allocator reuses these only after the launches
    return OrderedDict((k, results[k]) for k in keys)


def _extent(t: torch.Tensor) -> Tuple[int, int]:
    """[first byte, last byte + 1) of the memory a tensor's elements span."""
    span = 1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride())) if t.numel() else 0
    return t.data_ptr(), t.data_ptr() + span * t.element_size()


def _reads_running_sum(ts: Sequence[torch.Tensor]) -> List[int]:
    """Positions j >= 1 whose tensor IS client 0's (the same object or an
    identical view of its memory): FedAvg_seq / FedDyn add into client 0's
    tensor in place (agg_operator.py:58-63), so such an entry reads the running
    sum, not the original values.  A tensor that only partly overlaps client
    0's memory would read a mix of both; that is refused loudly."""
    t0 = ts[0]
    lo0, hi0 = _extent(t0)
    dev0 = t0.device
    pos = []
    for j in range(1, len(ts)):
        t = ts[j]
        if t is t0:
            pos.append(j)
            continue
        if t.device != dev0:
            continue
        lo, hi = _extent(t)
        if lo < hi0 and lo0 < hi:
            if (lo, hi) == (lo0, hi0) and t.stride() == t0.stride() and t.shape == t0.shape:
                pos.append(j)
            elif _shares_elements(t0, t):
                raise NotImplementedError(
                    f"client {j}'s tensor partly overlaps client 0's: the reference's in-place sum would read a "
                    "mix of running and original values, which fedml_amd does not reproduce")
            # else: interleaved views of one buffer that share no element (e.g.
            # clients holding different columns of one matrix) -- independent
    return pos


_OVERLAP_CHECK_MAX = 1 << 24  # elements: larger interleaved views are refused rather than enumerated


def _shares_elements(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Do two views whose byte extents overlap share an element?  Exact for
    views of one storage with element-aligned offsets (their element index
    sets are compared); anything else counts as sharing."""
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr() or a.element_size() != b.element_size():
        return True
    if a.numel() + b.numel() > _OVERLAP_CHECK_MAX:
        return True
    esz = a.element_size()
    base = a.untyped_storage().data_ptr()
    if (a.data_ptr() - base) % esz or (b.data_ptr() - base) % esz:
        return True

    def elements(t):
        off = (t.data_ptr() - base) // esz
        idx = torch.zeros((), dtype=torch.int64)
        for n, st in zip(t.shape, t.stride()):
            idx = idx.unsqueeze(-1) + torch.arange(n, dtype=torch.int64) * st
        return (idx.reshape(-1) + off).numpy()

    return bool(np.intersect1d(elements(a), elements(b)).size)


def sequential_sum_inplace(dicts: Sequence["OrderedDict"], keys: Sequence[str], args) -> None:
    """avg = p_0 ; avg += p_i, updating client 0's tensors in place
    (agg_operator.py:55-63, :68-77).  An entry that shares client 0's tensor
    (the same dict listed again, or the same tensor object) reads the running
    sum at its position, as the in-place `+=` makes it do in the reference:
    the chain is cut there and the next piece starts from [acc, acc, ...]."""
    per_key = _gather(dicts, keys)
    K = len(dicts)
    aliased: Dict[str, List[int]] = {}
    for k in keys:
        if K > 1 and per_key[k][0].numel():
            pos = _reads_running_sum(per_key[k])
            if pos:
                aliased[k] = pos
    plain = [k for k in keys if k not in aliased]
    _seq_sum_lists({k: per_key[k] for k in plain}, plain, K, args)
    for k, pos in aliased.items():
        ts = per_key[k]
        t0 = ts[0]
        head = ts[:pos[0]]
        _seq_sum_lists({k: head}, [k], len(head), args)
        for a, b in zip(pos, pos[1:] + [K]):
            seg = [t0, t0] + list(ts[a + 1:b])  # acc + acc, then the originals up to the next alias
            _seq_sum_lists({k: seg}, [k], len(seg), args)


def _seq_sum_lists(per_key: Dict[str, List[torch.Tensor]], keys: Sequence[str], K: int, args) -> None:
    """sum of per_key[k][0..K) into per_key[k][0], in place, in client order."""
    if K < 2:
        return
    staged = []
    for k in keys:
        ts = per_key[k]
        t0 = ts[0]
        if t0.numel() == 0:
            continue
        if t0.is_cuda and t0.dtype in _SUM_DTYPES and all(t.is_contiguous() for t in ts):
            device = t0.device
            with torch.cuda.device(device):  # in place, straight into client 0's tensor
                ptrs = [t.data_ptr() for t in ts]
                kn.sum_ptrs(t0.dtype, kn.upload_i64(ptrs, device), K, t0.numel(), t0, kn.aligned16(ptrs))
        else:
            staged.append(k)
    if not staged:
        return
    # host tensors (and exotic dtypes): rows in HBM, sum into row 0, copy back
    by_dev: Dict[torch.device, List[str]] = OrderedDict()
    for k in staged:
        t0 = per_key[k][0]
        by_dev.setdefault(t0.device if t0.is_cuda else _host_device(args), []).append(k)
    for device, dkeys in by_dev.items():
        with torch.cuda.device(device):
            bucket = ClientBucket([(k, tuple(per_key[k][0].shape), per_key[k][0].dtype) for k in dkeys], K, device,
                                  promote_ints=False)  # integer sums stay exact
            for i in range(K):
                bucket.put(i, {k: per_key[k][i] for k in dkeys}, 1)
            bucket.sync_ingest()
            for dt, g in bucket.groups.items():
                if g.length:
                    kn.sum_ptrs(dt, g.d_ptrs, K, g.length, g.rows[0], True)
            row0 = bucket.view(0)
            for k in dkeys:
                per_key[k][0].copy_(row0[k])  # dtype cast back (integer sums wrap like torch's)


# ---------------------------------------------------------------------------
# A dict listed more than once (agg_operator.py:36-44, :121-133)
#
# The reference's accumulator IS client 0's dict entry (`avg_params[k] = ...`
# at i == 0, then `+=`), so a later list entry that is the same dict object
# reads the running accumulator, not the original tensors (Mime: either of
# client 0's two dicts, in either role).  Such rounds run as a short program
# of ordinary weighted reductions: the client chain is cut wherever an entry
# reads a running accumulator, and the next piece starts from
# [acc (w = 1.0), acc (w = w_i), ...] -- fl(acc * 1.0) is acc exactly, so the
# pieces reproduce the reference's one chain bit for bit.


def _is_in(d, seq) -> int:
    for j, c in enumerate(seq):
        if d is c:
            return j
    return -1


def _reads_running_cell(raw_grad_list, roles: Sequence[int]) -> bool:
    """Does any step of the reference's loop read an accumulator it already
    wrote?  roles: the tuple positions of the accumulated dicts ((1,) FedAvg,
    (1, 2) Mime)."""
    written: List[object] = []
    for i in range(len(raw_grad_list)):
        for r in roles:
            if _is_in(raw_grad_list[i][r], written) >= 0:
                return True
            tgt = raw_grad_list[0][r]
            if _is_in(tgt, written) < 0:
                written.append(tgt)
    return False


def _reduce_chain(chain, keys: Sequence[str], args, reduce=None) -> "OrderedDict[str, torch.Tensor]":
    """One weighted chain over (dict, weight) sources.  A running value of an
    integer key is float32 (torch promotes `int * w`), so where a chain mixes
    it with original integer tensors those go in as fl32(v), which is what the
    kernel's int64 path computes with too."""
    dicts = [d for d, _ in chain]
    ws = [w for _, w in chain]
    mixed = set()
    for k in keys:
        dts = {d[k].dtype for d in dicts}
        if len(dts) > 1:
            mixed.add(k)
    if mixed:
        dicts = [OrderedDict((k, d[k].to(torch.float32) if k in mixed and not d[k].is_floating_point() else d[k])
                             for k in keys) for d in dicts]
    return (reduce or weighted_reduce)(dicts, keys, ws, args)


def _run_cells(raw_grad_list, roles: Sequence[int], keys: Sequence[str], weights: Sequence, args, reduce=None,
               one=1.0) -> None:
    """The reference's FedAvg / FedProx / Mime loop with its aliasing: cells
    are the accumulated dicts (client 0's), each step `cell = src * w`
    (i == 0) or `cell += src * w`, src read at that moment (a cell's running
    value if src is a cell already written).  Pending steps of a cell batch
    into one weighted reduction until another step reads it; the final values
    are bound into the cell dicts.  reduce / one: the chain's reduction and
    the weight that passes a running value through unchanged (muldiv_reduce
    with (1, 1) for the MPI simulation's order)."""
    cells: List[object] = []
    for r in roles:
        if _is_in(raw_grad_list[0][r], cells) < 0:
            cells.append(raw_grad_list[0][r])
    value: List[object] = [None] * len(cells)
    chain: List[object] = [None] * len(cells)
    written = [False] * len(cells)

    def flush(c: int) -> None:
        ch = chain[c]
        chain[c] = None
        if ch is None or (len(ch) == 1 and ch[0][0] is value[c] and ch[0][1] == one):
            return
        value[c] = _reduce_chain(ch, keys, args, reduce)

    for i in range(len(raw_grad_list)):
        w = weights[i]
        for r in roles:
            tc = _is_in(raw_grad_list[0][r], cells)
            src = raw_grad_list[i][r]
            sc = _is_in(src, cells)
            if sc >= 0 and written[sc]:
                flush(sc)
                src = value[sc]
            if i == 0:
                chain[tc] = [(src, w)]
            else:
                if chain[tc] is None:
                    chain[tc] = [(value[tc], one)]
                chain[tc].append((src, w))
            written[tc] = True
    for c in range(len(cells)):
        flush(c)
    for c, d in enumerate(cells):
        if written[c]:
            for k in keys:
                d[k] = value[c][k]


def torch_aggregator(args, raw_grad_list, training_num):
    """agg_operator.py:33-134, branch for branch."""
    opt = args.federated_optimizer
    K = len(raw_grad_list)
    if opt in ("FedAvg", "FedProx"):
        (num0, avg_params) = raw_grad_list[0]
        keys = list(avg_params.keys())
        if not keys:
            return avg_params
        weights = [raw_grad_list[i][0] / training_num for i in range(K)]  # ZeroDivisionError as :39
        if _reads_running_cell(raw_grad_list, (1,)):  # client 0's dict listed again
            _run_cells(raw_grad_list, (1,), keys, weights, args)
            return avg_params
        res = weighted_reduce([raw_grad_list[i][1] for i in range(K)], keys, weights, args)
        for k in keys:  # rebinds client 0's keys; its original tensors stay untouched
            avg_params[k] = res[k]
        return avg_params
    if opt in ("FedAvg_seq", "FedDyn"):
        (num0, avg_params) = raw_grad_list[0]
        keys = list(avg_params.keys())
        sequential_sum_inplace([raw_grad_list[i][1] for i in range(K)], keys, args)
        return avg_params
    if opt == "SCAFFOLD":
        (num0, total_weights_delta, total_c_delta_para) = raw_grad_list[0]
        keys = list(total_weights_delta.keys())
        _gather([raw_grad_list[i][1] for i in range(K)], keys)  # KeyError parity
        _gather([raw_grad_list[i][2] for i in range(K)], keys)
        _, weights_delta, c_delta_para = raw_grad_list[K - 1]
        weights = [raw_grad_list[i][0] / training_num for i in range(K)] if keys else []  # :107's ZeroDivisionError
        w_c = 1 / args.client_num_in_total
        firsts = [raw_grad_list[i][1] for i in range(K)]
        if any(_is_in(raw_grad_list[i][2], firsts) >= 0 for i in range(K)):
            raise NotImplementedError("SCAFFOLD: a dict used both as a weights delta and as a control variate")
        # :110,113: the running c_delta sum is client 0's own tensor (bound at
        # i == 0), so `+=` leaves Σ_i c_i in it, in place: the one side
        # effect of the branch that outlives it
        if K > 1:
            sequential_sum_inplace([raw_grad_list[i][2] for i in range(K)], keys, args)
        # :116-117 overwrite the weighted sums with the LAST client's delta and
        # its control variate times w_c; only that survives.
        scaled = weighted_reduce([c_delta_para], keys, [w_c], args)
        if weights_delta is total_weights_delta:
            # :116 binds the LAST client's entry, here client 0's dict itself
            # (always so at K = 1): the weighted chain of :111,114 (with its
            # aliasing) survives -- as float32 for integer keys
            _run_cells(raw_grad_list, (1,), keys, weights, args)
        for k in keys:
            total_weights_delta[k] = weights_delta[k]
            total_c_delta_para[k] = scaled[k]
        return (total_weights_delta, total_c_delta_para)
    if opt == "Mime":
        (num0, avg_params, avg_local_grad) = raw_grad_list[0]
        assert args.client_num_per_round == len(raw_grad_list)
        keys = list(avg_params.keys())
        weights = [raw_grad_list[i][0] / training_num for i in range(K)] if keys else []
        if keys and _reads_running_cell(raw_grad_list, (1, 2)):  # one of client 0's dicts listed again
            _run_cells(raw_grad_list, (1, 2), keys, weights, args)
            return (avg_params, avg_local_grad)
        res_p = weighted_reduce([raw_grad_list[i][1] for i in range(K)], keys, weights, args)
        res_g = weighted_reduce([raw_grad_list[i][2] for i in range(K)], keys, weights, args)
        for k in keys:
            avg_params[k] = res_p[k]
            avg_local_grad[k] = res_g[k]
        return (avg_params, avg_local_grad)
    # FedOpt / FedNova are `pass` in the reference (:64-67) and any other name
    # falls through: `return avg_params` then raises UnboundLocalError.  Server
    # optimizers live in fedml_amd.fedopt instead.
    raise UnboundLocalError("local variable 'avg_params' referenced before assignment")
