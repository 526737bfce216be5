"""Robust aggregation on MI355X: the two FedML defenses
that are pure reductions over the client axis.

"wise_median"   CoordinateWiseMedianDefense.defend_on_aggregation
                (core/security/defense/coordinate_wise_median_defense.py:18-44):
                stack the "weight" keys of every client (vectorize_weight,
                core/security/common/utils.py:8-21: all keys except BatchNorm
                running_mean / running_var / num_batches_tracked), take
                torch.median over clients per coordinate (lower median; NaN if
                the column has one), then walk client 0's keys ALL of them
                assigning consecutive slices of that vector (.view(size)).
                The walk is reproduced as is: for models with BN buffers the
                slices no longer line up with the weight keys and the last
                .view() raises RuntimeError — exactly what FedML does.
                The median itself is fedagg_median (one launch over the
                whole weight row; fp32 rows, or bf16 / f16 rows for 16-bit
                models, whose torch.cat stays 16-bit).

"trimmed_mean"  CoordinateWiseTrimmedMeanDefense.defend_before_aggregation
                (coordinate_wise_trimmed_mean_defense.py:19-26 ->
                common/utils.py:213-228 trimmed_mean): clients sorted by their
                sample count (compute_a_score), int(beta * K) dropped at each
                end, then ordinary FedAvg (our kernel) on the survivors.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Sequence, Tuple

import torch

from . import _native as nat
from . import kernels as kn
from .bucket import ClientBucket

DEFENSE_WISE_MEDIAN = "wise_median"
DEFENSE_TRIMMED_MEAN = "trimmed_mean"
SUPPORTED = (DEFENSE_WISE_MEDIAN, DEFENSE_TRIMMED_MEAN)


def is_weight_param(k: str) -> bool:
    """core/security/common/utils.py:16-21."""
    return "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k


def median_f32(d_ptrs: torch.Tensor, K: int, N: int, out: torch.Tensor) -> None:
    """Coordinate-wise lower median of K fp32 device rows (fedagg_median_f32)."""
    kn._require_cuda(out, "median_f32")
    nat.check(nat.lib().fedagg_median_f32(d_ptrs.data_ptr(), K, N, out.data_ptr(), 0, nat.stream_handle()),
              "median_f32")


_MEDIAN_DT = {torch.float32: nat.DT_F32, torch.bfloat16: nat.DT_BF16, torch.float16: nat.DT_F16}


def median_rows(d_ptrs: torch.Tensor, K: int, N: int, out: torch.Tensor, aligned: bool = False) -> None:
    """Coordinate-wise lower median of K device rows of out's dtype (fp32, bf16
    or f16; fedagg_median).  aligned: every row pointer and out are 16-byte
    aligned (bucket rows are), which lets 16-bit rows use the packed kernel."""
    kn._require_cuda(out, "median")
    if out.dtype not in _MEDIAN_DT:
        raise TypeError(f"median: fp32, bf16 or f16 rows (got {out.dtype})")
    flags = nat.FEDAGG_ALIGNED16 if aligned and out.data_ptr() % 16 == 0 else 0
    nat.check(nat.lib().fedagg_median(_MEDIAN_DT[out.dtype], d_ptrs.data_ptr(), K, N, out.data_ptr(), flags,
                                      nat.stream_handle()), "median")


def coordinate_wise_median(raw_client_grad_list: List[Tuple[float, "OrderedDict"]], device=None
                           ) -> "OrderedDict":
    """CoordinateWiseMedianDefense.defend_on_aggregation on the GPU."""
    K = len(raw_client_grad_list)
    dicts = [raw_client_grad_list[i][1] for i in range(K)]
    wkeys = [k for k in dicts[0].keys() if is_weight_param(k)]
    for d in dicts[1:]:
        for k in wkeys:
            d[k]  # KeyError for a missing key, as vectorize_weight would fail
    t0 = dicts[0][wkeys[0]] if wkeys else None
    if t0 is None:
        raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")  # vectorize_weight on no keys
    dev = t0.device if t0.is_cuda else (torch.device(device) if device is not None else
                                        torch.device("cuda", torch.cuda.current_device()))
    dts = {dicts[0][k].dtype for k in wkeys}
    # vectorize_weight's torch.cat promotes to one dtype: fp32 (with integer
    # weights riding as fl32(v)), or a 16-bit model's own bf16 / f16
    if dts <= {torch.float32, torch.int64, torch.int32, torch.bool} and torch.float32 in dts:
        row_dt = torch.float32
    elif dts in ({torch.bfloat16}, {torch.float16}):
        row_dt = next(iter(dts))
    else:
        raise NotImplementedError("wise_median on the GPU takes fp32 weights (integer keys allowed), or all-bf16 "
                                  f"/ all-f16 weights (got {sorted(map(str, dts))})")
    with torch.cuda.device(dev):
        layout = [(k, tuple(dicts[0][k].shape), dicts[0][k].dtype) for k in wkeys]
        bucket = ClientBucket(layout, K, dev)
        for i in range(K):
            bucket.put(i, {k: dicts[i][k] for k in wkeys}, 1)
        bucket.sync_ingest()
        g = bucket.groups[row_dt]
        row_med = torch.empty(g.padded, dtype=row_dt, device=dev)
        median_rows(g.d_ptrs, K, g.length, row_med, aligned=True)  # bucket rows are 256-B aligned
        # the reference's vector: weight keys back to back, no alignment gaps
        vec = torch.cat([row_med[o:o + n] for o, n in zip(g.offsets, g.numels)]) if g.keys else row_med[:0]
        if not t0.is_cuda:
            vec = vec.cpu()
    # coordinate_wise_median_defense.py:36-44: walk ALL of client 0's keys
    index = 0
    (num0, averaged_params) = raw_client_grad_list[0]
    for k, params in list(averaged_params.items()):
        median_params = vec[index:index + params.numel()].view(params.size())
        index += params.numel()
        averaged_params[k] = median_params
    return averaged_params


def compute_a_score(local_sample_number):
    """common/utils.py:231-233 (the score is the sample count)."""
    return local_sample_number


def trimmed_mean(model_list: Sequence, trimmed_num: int) -> list:
    """common/utils.py:213-228: a stable sort by score, then both ends dropped."""
    temp = [(n, grad, compute_a_score(n)) for n, grad in model_list]
    temp.sort(key=lambda x: x[2])
    temp = temp[trimmed_num: len(model_list) - trimmed_num]
    return [(t[0], t[1]) for t in temp]


def trimmed_mean_before_aggregation(raw_client_grad_list: Sequence, beta: float) -> list:
    """CoordinateWiseTrimmedMeanDefense.defend_before_aggregation (:19-26)."""
    if beta > 1 / 2 or beta < 0:
        raise ValueError("the bound of beta is [0, 1/2)")
    return trimmed_mean(raw_client_grad_list, int(beta * len(raw_client_grad_list)))
