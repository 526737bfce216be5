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
                models, whose torch.cat stays 16-bit; a mixed-width model's
                16-bit keys are widened into fp32 rows, as torch.cat promotes).

"trimmed_mean"  CoordinateWiseTrimmedMeanDefense.defend_before_aggregation
                (coordinate_wise_trimmed_mean_defense.py:19-26 ->
                common/utils.py:213-228 trimmed_mean): clients sorted by their
                sample count (compute_a_score), int(beta * K) dropped at each
                end, then ordinary FedAvg (our kernel) on the survivors.

"krum", "multikrum"
                KrumDefense.defend_before_aggregation (krum_defense.py:28-60):
                the K x K squared distances of the clients' weight vectors are
                one fedagg_pairdist2_f32 launch; the scores (sum of the
                K - f - 2 smallest), their fp32 argsort and the returned
                sub-list of the ORIGINAL (sample_num, dict) tuples follow the
                reference on the host (K numbers).

"slsgd"         SLSGDDefense (slsgd_defense.py:28-67): option 2 trims by
                sample count before aggregation (the trimmed-mean helper);
                on aggregation FedAvg, then (1 - alpha) g + alpha avg per key,
                a two-row weighted sum on the GPU (our FedAvg kernel: the
                same two roundings per element as torch).

"cclip"         CClipDefense (cclip_defense.py:21-80): bucketization =
                FedAvg over consecutive groups of bucket_size clients (our
                kernel, one launch per group), one bucket mean drawn by
                np.random.randint as the guess, each mean's distance to it
                (fedagg_dist2_f32), the scaled differences (mean - guess) *
                min(1, tau / dist) over every key (fedagg_scale_diff_f32);
                after aggregation guess + aggregate (a two-row sum).

"norm_diff_clipping"
                NormDiffClippingDefense.defend_before_aggregation
                (norm_diff_clipping_defense.py:20-54): every client's distance
                to the global model is one fedagg_dist2_f32 launch, the clipped
                weights (x - g) / max(1, norm / bound) + g one
                fedagg_clip_diff_f32 launch; non-weight keys stay the client's
                own tensors, as in the reference.

Distances: the reference forms fp32 differences and takes an fp32 torch.norm
(.item(), then ** 2 for Krum).  The kernels sum the exact squares of the same
fp32 differences in fp64; the host rounds the root to fp32 as the reference's
norm does.  torch's own fp32 reduction may land one ulp away from that, so a
Krum selection matches the reference's except between clients whose fp32
scores are within an ulp (exact ties, e.g. mirror-image clients, can go either
way in the reference too: its reduction order depends on the thread count),
and a clipped client's divisor can differ in its last bit.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _native as nat
from . import kernels as kn
from .bucket import ClientBucket

DEFENSE_WISE_MEDIAN = "wise_median"
DEFENSE_TRIMMED_MEAN = "trimmed_mean"
DEFENSE_KRUM = "krum"
DEFENSE_MULTIKRUM = "multikrum"
DEFENSE_NORM_DIFF_CLIPPING = "norm_diff_clipping"
DEFENSE_SLSGD = "slsgd"
DEFENSE_CCLIP = "cclip"
DEFENSE_ROBUST_LEARNING_RATE = "robust_learning_rate"
DEFENSE_WEAK_DP = "weak_dp"
SUPPORTED = (DEFENSE_WISE_MEDIAN, DEFENSE_TRIMMED_MEAN, DEFENSE_KRUM, DEFENSE_MULTIKRUM, DEFENSE_NORM_DIFF_CLIPPING,
             DEFENSE_SLSGD, DEFENSE_CCLIP, DEFENSE_ROBUST_LEARNING_RATE, DEFENSE_WEAK_DP)
# FedMLDefender constructs these but lists them under none of its
# before / on / after-aggregation hooks (fedml_defender.py:131-154), so the
# plugin path aggregates as if no defense were set; they act only through
# FedMLDefender.defend (the MPI FedAvg aggregator)
PLUGIN_IDENTITY = (DEFENSE_ROBUST_LEARNING_RATE, DEFENSE_WEAK_DP)


def is_weight_param(k: str) -> bool:
    """core/security/common/utils.py:16-21."""
    return "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k


def _one_device(d0, wkeys, what: str) -> None:
    """The defenses gather every client's weight keys into one bucket on one
    GPU.  A round that a MultiDeviceBucket spread over several GPUs (because
    it did not fit one) would be pulled back onto one device and fail with an
    out-of-memory error deep inside; say what happened instead."""
    devs = {d0[k].device for k in wkeys if isinstance(d0[k], torch.Tensor) and d0[k].is_cuda}
    if len(devs) > 1:
        raise NotImplementedError(
            f"{what}: the clients' weight keys are spread over {len(devs)} GPUs "
            f"({', '.join(sorted(str(d) for d in devs))}; a multi-device round, fedml_amd.multidev); the defense "
            f"gathers every client onto one GPU, so run it on a round that fits one device")


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


def median_row_dtype(dts) -> torch.dtype:
    """The dtype of the median's rows for weight keys of dtypes `dts`:
    vectorize_weight's torch.cat promotes to one dtype, fp32 when any key is
    fp32 or two float widths meet (bf16 + f16 -> fp32; the 16-bit keys widen
    exactly, integer weights ride as fl32(v)), or a 16-bit model's own bf16 /
    f16.  The median is one of its inputs, so selecting in the promoted dtype
    is exact.  Other mixes (all-integer, 16-bit floats with integers) raise."""
    dts = set(dts)
    floats = dts & {torch.float32, torch.bfloat16, torch.float16}
    ints = dts - floats
    if (torch.float32 in floats or len(floats) > 1) and ints <= {torch.int64, torch.int32, torch.bool}:
        return torch.float32
    if dts in ({torch.bfloat16}, {torch.float16}):
        return next(iter(dts))
    raise NotImplementedError("wise_median on the GPU takes fp32 or mixed-width float weights (integer keys "
                              f"allowed), or all-bf16 / all-f16 weights (got {sorted(map(str, dts))})")


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
    _one_device(dicts[0], wkeys, "wise_median")
    dev = t0.device if t0.is_cuda else (torch.device(device) if device is not None else
                                        torch.device("cuda", torch.cuda.current_device()))
    dts = {dicts[0][k].dtype for k in wkeys}
    row_dt = median_row_dtype(dts)
    floats = dts & {torch.float32, torch.bfloat16, torch.float16}
    with torch.cuda.device(dev):
        # 16-bit keys of a promoted model are declared fp32: put() widens them
        layout = [(k, tuple(dicts[0][k].shape),
                   row_dt if dicts[0][k].dtype in floats else dicts[0][k].dtype) for k in wkeys]
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


# ---- distance-based defenses (csrc/robust.hip) ---------------------------------

def weight_chunks(group, chunk: int, device, absolute: bool = True) -> Tuple[torch.Tensor, int]:
    """Device (start, length) table of a row group's weight-key columns, runs
    of adjacent keys merged, split into pieces of at most `chunk` columns.

    absolute (default): cut at multiples of `chunk` in the row (a run's first
    piece is shorter), so pieces after the first start on whole cache lines.
    The kernels hand consecutive pieces to blocks on different XCDs; runs cut
    from their 16-byte aligned start made every boundary line a fetch for
    both blocks: dist2 at 1.036x the algorithmic bytes (1.009x now), Krum's
    Gram 5.58 ms (5.39 now) at config 3.  False: cuts from each run's start
    (tools' A/B baseline)."""
    segs = []
    for key, off, n in zip(group.keys, group.offsets, group.numels):
        if n == 0 or not is_weight_param(key):
            continue
        if segs and segs[-1][0] + segs[-1][1] == off:
            segs[-1][1] += n
        else:
            segs.append([off, n])
    starts, lens = [], []
    for off, n in segs:
        if absolute:
            st = np.concatenate([np.array([off], dtype=np.int64),
                                 np.arange((off // chunk + 1) * chunk, off + n, chunk, dtype=np.int64)])
        else:
            st = np.arange(off, off + n, chunk, dtype=np.int64)
        starts.append(st)
        lens.append(np.append(st[1:], off + n) - st)
    if not starts:
        return torch.zeros(2, dtype=torch.int64, device=device), 0
    tab = np.stack([np.concatenate(starts), np.concatenate(lens)], axis=1).ravel()
    return kn.upload_i64(tab.tolist(), device), len(tab) // 2


def _work(kind: int, K: int, n_chunks: int, device) -> torch.Tensor:
    n = int(nat.lib().fedagg_robust_work_len(kind, K, n_chunks))
    if n < 0:
        raise nat.FedAggNativeError("fedagg_robust_work_len: bad sizes")
    return torch.empty(max(n, 1), dtype=torch.float64, device=device)


GRAM_MAX_CLIENTS = 128  # fedagg_pairgram2_f32 holds up to 128 clients
# "auto" keeps the Gram's distances only while (|c_i|^2 + |c_j|^2) / D_ij stays
# at or below this for every pair (c = the rows centred on the client mean):
# iid clients sit near 1; one update scaled far away inflates every honest
# client's |c|^2 and triggers the exact kernel (gram_condition)
GRAM_MAX_CONDITION = 8.0


def gram_condition(D: np.ndarray) -> float:
    """max over client pairs i != j of (|c_i|^2 + |c_j|^2) / D_ij, where c_i is
    client i's row minus the mean of the K rows: the factor by which the
    centred Gram's rounding error (~1e-7 (|c_i|^2 + |c_j|^2) per entry) exceeds
    a relative error of D_ij itself.  The centred norms come from D alone
    (double centring of a squared-distance matrix: |c_i|^2 = mean_j D_ij -
    sum D / (2 K^2)).  inf when two distinct clients are at distance 0, or when any distance
    or centred norm is not finite (an inf client, squares beyond fp32)."""
    K = D.shape[0]
    if K < 2:
        return 0.0
    D = np.asarray(D, dtype=np.float64)
    if not np.all(np.isfinite(D)):  # an inf / NaN client, or squares beyond fp32: only the exact kernel copes
        return float("inf")
    c2 = np.maximum(D.sum(axis=1) / K - D.sum() / (2.0 * K * K), 0.0)
    if not np.all(np.isfinite(c2)):
        return float("inf")
    num = c2[:, None] + c2[None, :]
    off = ~np.eye(K, dtype=bool)
    d, s = D[off], num[off]
    if np.any((d <= 0) & (s > 0)):
        return float("inf")
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(d > 0, s / np.where(d > 0, d, 1.0), 0.0)
    m = float(r.max())
    return m if np.isfinite(m) else float("inf")


def pairdist2_rows(d_ptrs: torch.Tensor, K: int, chunks: torch.Tensor, n_chunks: int, device,
                   method: str = "auto") -> torch.Tensor:
    """K x K fp64 squared distances of K fp32 device rows over the chunked
    columns.  method "exact": the reference's fp32 differences, squared and
    summed on the VALU (fedagg_pairdist2_f32); "gram": the centred Gram on the
    bf16 matrix cores with an exact three-way split (fedagg_pairgram2_f32,
    K <= 128); "auto": gram when K allows it (same Krum
    selections, ~3x faster at config 3)
    and the result is well conditioned (``gram_condition`` <=
    GRAM_MAX_CONDITION), else the exact kernel: one far-away update (the case
    Krum exists for) moves the client mean, and the honest clients' distances
    would then carry the Gram's error scaled by that update's norm."""
    if method not in ("auto", "gram", "exact"):
        raise ValueError(f"pair distance method {method!r}: 'auto', 'gram' or 'exact'")
    gram = method == "gram" or (method == "auto" and K <= GRAM_MAX_CLIENTS)
    if gram and K > GRAM_MAX_CLIENTS:
        raise ValueError(f"the Gram pair kernel holds at most {GRAM_MAX_CLIENTS} clients (K = {K})")
    out = torch.empty((K, K), dtype=torch.float64, device=device)
    work = _work(nat.WORK_PAIRGRAM if gram else nat.WORK_PAIRDIST2, K, n_chunks, device)
    fn = nat.lib().fedagg_pairgram2_f32 if gram else nat.lib().fedagg_pairdist2_f32
    nat.check(fn(d_ptrs.data_ptr(), K, chunks.data_ptr(), n_chunks, out.data_ptr(), work.data_ptr(), work.numel(),
                 nat.stream_handle()), "pairgram2" if gram else "pairdist2")
    if gram and method == "auto" and gram_condition(out.cpu().numpy()) > GRAM_MAX_CONDITION:
        return pairdist2_rows(d_ptrs, K, chunks, n_chunks, device, "exact")
    return out


def dist2_rows(d_ptrs: torch.Tensor, K: int, ref: "torch.Tensor | None", chunks: torch.Tensor, n_chunks: int,
               device) -> torch.Tensor:
    """K fp64 squared distances of K fp32 device rows to `ref` (None: norms)
    over the chunked columns (fedagg_dist2_f32)."""
    out = torch.empty(K, dtype=torch.float64, device=device)
    work = _work(nat.WORK_DIST2, K, n_chunks, device)
    nat.check(nat.lib().fedagg_dist2_f32(d_ptrs.data_ptr(), K, ref.data_ptr() if ref is not None else None,
                                         chunks.data_ptr(), n_chunks, out.data_ptr(), work.data_ptr(),
                                         work.numel(), nat.stream_handle()), "dist2")
    return out


def fp32_norm(sq: float) -> float:
    """The reference's `torch.norm(fp32 vector).item()`: an fp32 root."""
    return float(np.float32(np.sqrt(sq)))


def _weight_bucket(dicts: Sequence, what: str, device=None):
    """ClientBucket of the clients' weight keys (vectorize_weight's keys, in
    client 0's order) and its fp32 row group."""
    wkeys = [k for k in dicts[0].keys() if is_weight_param(k)]
    if not wkeys:
        raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")  # vectorize_weight on no keys
    for d in dicts[1:]:
        for k in wkeys:
            d[k]  # KeyError for a missing key, as the reference's walk would fail
    dts = {dicts[0][k].dtype for k in wkeys}
    if dts != {torch.float32}:
        raise NotImplementedError(f"{what} on the GPU takes fp32 weight keys (got {sorted(map(str, dts))})")
    _one_device(dicts[0], wkeys, what)
    t0 = dicts[0][wkeys[0]]
    dev = t0.device if t0.is_cuda else (torch.device(device) if device is not None else
                                        torch.device("cuda", torch.cuda.current_device()))
    layout = [(k, tuple(dicts[0][k].shape), torch.float32) for k in wkeys]
    with torch.cuda.device(dev):
        bucket = ClientBucket(layout, len(dicts), dev)
        for i, d in enumerate(dicts):
            bucket.put(i, {k: d[k] for k in wkeys}, 1)
        bucket.sync_ingest()
    return bucket, bucket.groups[torch.float32], wkeys, dev


def krum_scores(D: np.ndarray, byzantine_client_num: int) -> list:
    """KrumDefense._compute_krum_score (krum_defense.py:47-60) over the K x K
    squared distances: each distance enters as the reference's
    `norm.item() ** 2`, the K - f - 2 smallest are summed in ascending order."""
    K = D.shape[0]
    scores = []
    for i in range(K):
        dists = [fp32_norm(D[i, j]) ** 2 for j in range(K) if j != i]
        dists.sort()
        scores.append(sum(dists[0:K - byzantine_client_num - 2]))
    return scores


def krum_before_aggregation(raw_client_grad_list: Sequence, byzantine_client_num: int, krum_param_m: int = 1,
                            device=None, method: str = "auto") -> list:
    """KrumDefense.defend_before_aggregation (krum_defense.py:28-45): the
    krum_param_m lowest-scoring clients' original tuples, in score order.
    method: the pair-distance kernel (pairdist2_rows)."""
    num_client = len(raw_client_grad_list)
    if not 2 * byzantine_client_num + 2 <= num_client - krum_param_m:
        raise ValueError("byzantine_client_num conflicts with requirements in Krum: "
                         "2 * byzantine_client_num + 2 < client number - krum_param_m")
    bucket, g, _, dev = _weight_bucket([item[1] for item in raw_client_grad_list], "krum", device)
    with torch.cuda.device(dev):
        chunks, n_chunks = weight_chunks(g, nat.PAIR_CHUNK, dev)
        D = pairdist2_rows(g.d_ptrs, num_client, chunks, n_chunks, dev, method).cpu().numpy()
    scores = krum_scores(D, byzantine_client_num)
    score_index = torch.argsort(torch.Tensor(scores)).tolist()[0:krum_param_m]
    return [raw_client_grad_list[i] for i in score_index]


def krum_param_m(args) -> int:
    """KrumDefense.__init__ (krum_defense.py:19-25)."""
    m = getattr(args, "krum_param_m", None)
    return m if isinstance(m, int) else 1


def norm_diff_clipping_before_aggregation(raw_client_grad_list: Sequence, global_model, norm_bound: float,
                                          device=None) -> list:
    """NormDiffClippingDefense.defend_before_aggregation
    (norm_diff_clipping_defense.py:20-54): every client's weights pulled to
    within norm_bound of the global model; new dicts, the client's own
    tensors for non-weight keys."""
    K = len(raw_client_grad_list)
    if K == 0:
        return []
    dicts = [item[1] for item in raw_client_grad_list]
    bucket, g, wkeys, dev = _weight_bucket(dicts, "norm_diff_clipping", device)
    with torch.cuda.device(dev):
        gb = ClientBucket([(k, tuple(dicts[0][k].shape), torch.float32) for k in wkeys], 1, dev)
        gb.put(0, {k: global_model[k] for k in wkeys}, 1)
        gb.sync_ingest()
        ref = gb.groups[torch.float32].rows[0]
        chunks, n_chunks = weight_chunks(g, nat.DIST_CHUNK, dev)
        sq = dist2_rows(g.d_ptrs, K, ref, chunks, n_chunks, dev).cpu().numpy()
        divs = [max(1, fp32_norm(s) / norm_bound) for s in sq]  # _get_clipped_norm_diff
        d_div = kn.upload_f32(divs, dev)
        out = torch.empty_like(g.rows)
        d_dst = kn.upload_i64([out[i].data_ptr() for i in range(K)], dev)
        nat.check(nat.lib().fedagg_clip_diff_f32(g.d_ptrs.data_ptr(), K, ref.data_ptr(), d_div.data_ptr(),
                                                 g.rows.shape[1], d_dst.data_ptr(), nat.stream_handle()),
                  "clip_diff")
        if not dicts[0][wkeys[0]].is_cuda:
            out = out.cpu()  # host clients get host tensors back, as the reference returns
        else:
            torch.cuda.current_stream().synchronize()  # the staging buckets go out of scope
    pos = {k: j for j, k in enumerate(g.keys)}
    new_list = []
    for i, (sample_num, local_w) in enumerate(raw_client_grad_list):
        clipped = OrderedDict()
        for k, v in local_w.items():  # _get_clipped_weights (:44-54)
            if is_weight_param(k):
                j = pos[k]
                clipped[k] = out[i, g.offsets[j]:g.offsets[j] + g.numels[j]].view(v.size())
            else:
                clipped[k] = v
        new_list.append((sample_num, clipped))
    return new_list


# ---- SLSGD / CClip (two-row and grouped weighted sums, scaled differences) ------

def _like_input(out: "OrderedDict[str, torch.Tensor]", on_device: bool) -> "OrderedDict[str, torch.Tensor]":
    if on_device:
        return out
    return OrderedDict((k, t.cpu()) for k, t in out.items())


def _float_bucket(template, capacity: int, what: str, device=None):
    """A ClientBucket for fp32 models (integer buffers allowed: they sit in
    the fp32 row as fl32(v), the dtype torch's int64 * float yields), laid out
    by `template`'s keys, on its device (or `device` for host tensors)."""
    keys = list(template.keys())
    layout = [(k, tuple(template[k].shape), template[k].dtype) for k in keys]
    dts = {dt for _, _, dt in layout}
    if not dts <= {torch.float32, torch.int64, torch.int32} or torch.float32 not in dts:
        raise NotImplementedError(f"{what} on the GPU takes fp32 models (integer buffers allowed), got "
                                  f"{sorted(map(str, dts))}")
    t0 = template[keys[0]]
    dev = t0.device if t0.is_cuda else (torch.device(device) if device is not None else
                                        torch.device("cuda", torch.cuda.current_device()))
    with torch.cuda.device(dev):
        bucket = ClientBucket(layout, capacity, dev)
    return bucket, dev


def _put_float(bucket, slot: int, d, keys) -> None:
    """put() of the layout's keys; an integer tensor under a float key is
    converted by put (fl32(v), torch's rounding of int64 -> float32)."""
    bucket.put(slot, OrderedDict((k, d[k]) for k in keys), 1)


def mix_two(first, second, w_first: float, w_second: float, device=None) -> "OrderedDict[str, torch.Tensor]":
    """fl(w_first * first[k]) + fl(w_second * second[k]) for every key of
    `second`, as torch computes `(1 - alpha) * g[k] + alpha * avg[k]` (two
    rows of our weighted-sum kernel; integer keys enter as fl32(v))."""
    keys = list(second.keys())
    on_dev = second[keys[0]].is_cuda
    bucket, dev = _float_bucket(second, 2, "slsgd / cclip", device)
    with torch.cuda.device(dev):
        _put_float(bucket, 0, first, keys)
        _put_float(bucket, 1, second, keys)
        bucket.sync_ingest()
        outs = bucket.new_outputs()
        bucket.reduce_into(outs, [w_first, w_second], 2)
        res = OrderedDict((k, t.clone()) for k, t in bucket.unflatten(outs).items())
    return _like_input(res, on_dev)


def slsgd_alpha_check(alpha: float) -> None:
    """SLSGDDefense.__init__ (slsgd_defense.py:29-33)."""
    if alpha > 1 or alpha < 0:
        raise ValueError("the bound of alpha is [0, 1]")


def slsgd_before_aggregation(raw_client_grad_list: Sequence, b: int, option_type: int) -> list:
    """SLSGDDefense.defend_before_aggregation (slsgd_defense.py:36-52)."""
    if b > math.ceil(len(raw_client_grad_list) / 2) - 1 or b < 0:
        raise ValueError("the bound of b is [0, {}])".format(math.ceil(len(raw_client_grad_list) / 2) - 1))
    if option_type != 1 and option_type != 2:
        raise Exception("Such option type does not exist!")
    if option_type == 2:
        raw_client_grad_list = trimmed_mean(raw_client_grad_list, b)
    return list(raw_client_grad_list)


def slsgd_on_aggregation(avg_params, global_model, alpha: float, device=None):
    """SLSGDDefense.defend_on_aggregation (slsgd_defense.py:54-67) after the
    base FedAvg: (1 - alpha) * global + alpha * avg for every key."""
    return mix_two(global_model, avg_params, 1 - alpha, alpha, device)


def cclip_tau(args) -> float:
    """CClipDefense.__init__ (cclip_defense.py:22-26)."""
    tau = getattr(args, "tau", None)
    return tau if type(tau) in [int, float] and tau > 0 else 10


def cclip_before_aggregation(raw_client_grad_list: Sequence, tau: float, bucket_size: int, device=None):
    """CClipDefense.defend_before_aggregation (cclip_defense.py:30-56).
    Returns (new list, initial guess dict) -- the guess is kept for
    defend_after_aggregation, as the reference's defender object does."""
    K = len(raw_client_grad_list)
    dicts = [item[1] for item in raw_client_grad_list]
    on_dev = next(iter(dicts[0].values())).is_cuda
    bucket, dev = _float_bucket(dicts[0], K, "cclip", device)
    keys = list(dicts[0].keys())
    with torch.cuda.device(dev):
        for i, d in enumerate(dicts):
            bucket.put(i, {k: d[k] for k in keys}, 1)
        bucket.sync_ingest()
    g = bucket.groups[torch.float32]
    B = math.ceil(K / bucket_size)
    with torch.cuda.device(dev):
        means = torch.empty((B, g.rows.shape[1]), dtype=torch.float32, device=dev)
        nums = []
        for b in range(B):  # Bucket.bucketization (common/bucket.py:6-28)
            lo = b * bucket_size
            cn = min(bucket_size, K - lo)
            sample_num = 0
            for i in range(cn):
                sample_num += raw_client_grad_list[lo + i][0]
            w = [raw_client_grad_list[lo + i][0] / sample_num for i in range(cn)]
            kn.wsum_ptrs(torch.float32, g.d_ptrs[lo:lo + cn], kn.weights_for(w, torch.float32, dev), cn, g.length,
                         means[b], True)
            nums.append(sample_num)
        guess_idx = np.random.randint(0, B)  # _compute_an_initial_guess (:61-62), the global numpy RNG
        guess = means[guess_idx]
        m_ptrs = kn.upload_i64([means[b].data_ptr() for b in range(B)], dev)
        chunks, n_chunks = weight_chunks(g, nat.DIST_CHUNK, dev)
        sq = dist2_rows(m_ptrs, B, guess, chunks, n_chunks, dev).cpu().numpy()
        scores = [min(1, tau / (fp32_norm(v) + 1e-8)) for v in sq]  # _compute_cclip_score (:64-71)
        d_sc = kn.upload_f32([float(x) for x in scores], dev)
        out = torch.empty_like(means)
        d_dst = kn.upload_i64([out[b].data_ptr() for b in range(B)], dev)
        nat.check(nat.lib().fedagg_scale_diff_f32(m_ptrs.data_ptr(), B, guess.data_ptr(), d_sc.data_ptr(),
                                                  g.rows.shape[1], d_dst.data_ptr(), nat.stream_handle()),
                  "scale_diff")
        views = [bucket_view(g, out[b]) for b in range(B)]
        guess_dict = bucket_view(g, guess)
    new_list = [(nums[b], _like_input(views[b], on_dev)) for b in range(B)]
    return new_list, _like_input(guess_dict, on_dev)


def bucket_view(group, row: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
    """Per-key views of one fp32 row of a group (keys in layout order)."""
    return OrderedDict((k, row[o:o + n].view(shp))
                       for k, o, n, shp in zip(group.keys, group.offsets, group.numels, group.shapes))


def cclip_after_aggregation(global_model, initial_guess, device=None):
    """CClipDefense.defend_after_aggregation (cclip_defense.py:57-60):
    guess[k] + global[k] for every key (a two-row sum, weights 1 and 1:
    fl(1 * x) = x, so one rounding, as torch's add)."""
    return mix_two(initial_guess, global_model, 1.0, 1.0, device)


# ---- Robust learning rate (sign agreement per coordinate) ----------------------

def robust_learning_rate(raw_client_grad_list: Sequence, robust_threshold, base_aggregation_func=None,
                         device=None) -> "OrderedDict[str, torch.Tensor]":
    """RobustLearningRateDefense.run (robust_learning_rate_defense.py:35-62) on
    the GPU: ONE pass over the clients' rows computes the FedAvg chain and the
    per-coordinate sum of their signs (fedagg_wsum_rlr_f32), and the key
    becomes lr * avg with lr = +1 where |Σ sign| >= threshold, else -1.
    As in the reference: threshold 0 hands the list to base_aggregation_func,
    the weights are n_i / Σn (ZeroDivisionError at Σn = 0), a missing key
    raises KeyError, and client 0's dict is returned with its keys rebound
    (integer keys come back fp32: torch's fp32 average times the integer lr)."""
    if robust_threshold == 0:
        return base_aggregation_func(raw_client_grad_list)
    total = 0
    for n, _ in raw_client_grad_list:
        total += n
    K = len(raw_client_grad_list)
    ws = [n / total for n, _ in raw_client_grad_list]
    num0, avg_params = raw_client_grad_list[0]
    keys = list(avg_params.keys())
    on_dev = avg_params[keys[0]].is_cuda
    bucket, dev = _float_bucket(avg_params, K, "robust_learning_rate", device)
    with torch.cuda.device(dev):
        for i, (_, d) in enumerate(raw_client_grad_list):
            _put_float(bucket, i, d, keys)
        bucket.sync_ingest()
        outs = bucket.new_outputs()
        g = bucket.groups[torch.float32]
        kn.wsum_rlr_ptrs(g.d_ptrs, kn.weights_for(ws, torch.float32, dev), K, g.length,
                         float(np.float32(robust_threshold)), outs[torch.float32], True)
        res = _like_input(OrderedDict((k, t.clone()) for k, t in bucket.unflatten(outs).items()), on_dev)
    for k in keys:
        avg_params[k] = res[k]
    return avg_params


class RobustLearningRateDefense:
    """Drop-in for FedML's RobustLearningRateDefense (the object
    FedMLDefender.init builds for defense_type "robust_learning_rate"):
    FedMLDefender.defend -> run() aggregates on the GPU."""

    def __init__(self, config):
        self.robust_threshold = config.robust_threshold
        self.server_learning_rate = 1

    def run(self, raw_client_grad_list, base_aggregation_func=None, extra_auxiliary_info=None):
        return robust_learning_rate(raw_client_grad_list, self.robust_threshold, base_aggregation_func)

    def defend_before_aggregation(self, raw_client_grad_list, extra_auxiliary_info=None):
        return None  # BaseDefenseMethod's default (defense_base.py:11-24)

    def defend_on_aggregation(self, raw_client_grad_list, base_aggregation_func=None, extra_auxiliary_info=None):
        return None

    def get_malicious_client_idxs(self):
        return []
