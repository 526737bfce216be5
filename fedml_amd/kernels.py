"""Thin typed wrappers over the C ABI (include/fedagg.h) for torch tensors.

Every function here launches on the CURRENT torch stream of the tensors'
device and returns without synchronising.  Pointer tables and weight vectors
are uploaded from pinned host memory on that same stream, so they are
stream-ordered with the kernel that reads them.  There is no CPU fallback:
non-CUDA tensors raise.
"""
from __future__ import annotations

import array
import ctypes
import functools
import operator
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as nat

_DT_CODE = {torch.float32: nat.DT_F32, torch.bfloat16: nat.DT_BF16, torch.float16: nat.DT_F16,
            torch.float64: nat.DT_F64, torch.int64: nat.DT_I64, torch.int32: nat.DT_I32}

ACC_REFERENCE = nat.FEDAGG_ACC_REFERENCE
ACC_FP32 = nat.FEDAGG_ACC_FP32


def _require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise nat.FedAggNativeError(f"{what}: expected a device tensor, got {t.device} (no CPU fallback)")


_CUDA: list = []  # torch.cuda.is_available(), asked once (it reads the environment on every call)


def _cuda_ok() -> bool:
    if not _CUDA:
        _CUDA.append(torch.cuda.is_available())
    return _CUDA[0]


def upload_i64(values: Sequence[int], device: torch.device) -> torch.Tensor:
    arr = np.asarray(values, dtype=np.int64)  # ~2x faster than torch.tensor(list) on 40k pointers
    if _cuda_ok():
        host = torch.empty(arr.shape, dtype=torch.int64, pin_memory=True)
        host.numpy()[...] = arr
    else:
        host = torch.from_numpy(arr)
    return host.to(device, non_blocking=True)


def upload_f32(values: Sequence[float], device: torch.device) -> torch.Tensor:
    host = torch.tensor([float(v) for v in values], dtype=torch.float32)
    if _cuda_ok():
        host = host.pin_memory()
    return host.to(device, non_blocking=True)


def upload_f64(values: Sequence[float], device: torch.device) -> torch.Tensor:
    host = torch.tensor([float(v) for v in values], dtype=torch.float64)
    if _cuda_ok():
        host = host.pin_memory()
    return host.to(device, non_blocking=True)


INLINE_MAX_K = 256  # FEDAGG_HOST_WEIGHTS limit (include/fedagg.h)


class HostWeights:
    """Weights handed to a launch BY VALUE (kernel arguments): no upload, no
    device buffer.  Only for K <= INLINE_MAX_K."""

    def __init__(self, values: Sequence[float], dtype: torch.dtype = torch.float32):
        if len(values) > INLINE_MAX_K:
            raise ValueError(f"host weights need K <= {INLINE_MAX_K}")
        ct = ctypes.c_double if dtype == torch.float64 else ctypes.c_float
        self.buf = (ct * max(1, len(values)))(*[float(v) for v in values])

    def data_ptr(self) -> int:
        return ctypes.addressof(self.buf)


_LAST_HOST_W: dict = {}  # per weight dtype: (values' bytes, HostWeights) of the last ones built


def weights_for(values: Sequence[float], dtype: torch.dtype, device: torch.device):
    """Kernel-argument weights when K allows, else a device array.

    The last HostWeights built is reused for the same values (keyed by their
    exact fp64 bytes, so -0.0 and NaN payloads are told apart): a round over
    G shards or several dtype groups builds it once.  The launch copies the
    values into the kernel arguments, and nothing writes a HostWeights after
    construction, so sharing one is safe."""
    wdt = torch.float64 if dtype == torch.float64 else torch.float32
    if len(values) <= INLINE_MAX_K:
        key = array.array("d", values).tobytes()
        last = _LAST_HOST_W.get(wdt)
        if last is not None and last[0] == key:
            return last[1]
        hw = HostWeights(values, wdt)
        _LAST_HOST_W[wdt] = (key, hw)
        return hw
    return upload_f64(values, device) if wdt == torch.float64 else upload_f32(values, device)


def aligned16(ptrs: Sequence[int]) -> bool:
    return (functools.reduce(operator.or_, ptrs, 0) & 15) == 0


def wsum_rlr_ptrs(d_ptrs: torch.Tensor, d_w, K: int, N: int, threshold: float, out: torch.Tensor,
                  aligned: bool) -> None:
    """fedagg_wsum_rlr_f32: the FedAvg chain and the robust-learning-rate sign
    rule over K fp32 sources in one pass (RobustLearningRateDefense.run)."""
    _require_cuda(out, "wsum_rlr")
    if out.dtype != torch.float32:
        raise TypeError("robust learning rate: fp32 rows and output")
    flags = nat.FEDAGG_ALIGNED16 if aligned and (out.data_ptr() & 15) == 0 else 0
    if isinstance(d_w, HostWeights):
        flags |= nat.FEDAGG_HOST_WEIGHTS
    nat.check(nat.lib().fedagg_wsum_rlr_f32(d_ptrs.data_ptr(), d_w.data_ptr(), K, N, float(threshold),
                                            out.data_ptr(), flags, nat.stream_handle()), "wsum_rlr")


def wsum_ptrs(dtype: torch.dtype, d_ptrs: torch.Tensor, d_w: torch.Tensor, K: int, N: int,
              out: torch.Tensor, aligned: bool, acc_mode: int = ACC_REFERENCE, stream: Optional[int] = None) -> None:
    """Weighted sum over K sources given as a device pointer table; on the
    current stream, or on the raw hipStream_t `stream`."""
    _require_cuda(out, "wsum")
    if N == 0:  # empty keys: nothing to launch (their outputs may have no storage)
        return
    lib = nat.lib()
    st = stream if stream is not None else nat.stream_handle()
    flags = nat.FEDAGG_ALIGNED16 if aligned and (out.data_ptr() & 15) == 0 else 0
    if isinstance(d_w, HostWeights):
        flags |= nat.FEDAGG_HOST_WEIGHTS
    a = (d_ptrs.data_ptr(), d_w.data_ptr(), K, N, out.data_ptr())
    if dtype == torch.float32:
        if out.dtype == torch.float32:
            rc = lib.fedagg_wsum_f32(*a, flags, st)
        else:
            raise TypeError("fp32 sources produce fp32")
    elif dtype == torch.bfloat16:
        if out.dtype == torch.bfloat16:
            rc = lib.fedagg_wsum_bf16(*a, acc_mode, flags, st)
        elif out.dtype == torch.float32:
            rc = lib.fedagg_wsum_bf16_f32out(*a, flags, st)
        else:
            raise TypeError("bf16 sources produce bf16 or an fp32 partial")
    elif dtype == torch.float16:
        rc = lib.fedagg_wsum_f16(*a, acc_mode, flags, st)
    elif dtype == torch.float64:
        rc = lib.fedagg_wsum_f64(*a, flags, st)
    elif dtype == torch.int64:
        rc = lib.fedagg_wsum_i64_f32(*a, flags, st)
    else:
        raise TypeError(f"wsum: unsupported dtype {dtype}")
    nat.check(rc, f"wsum[{dtype}]")


_MULDIV_F = np.dtype([("n", "<f4"), ("d", "<f4")])
_MULDIV_D = np.dtype([("n", "<f8"), ("d", "<f8")])
_MULDIV_I = np.dtype([("n", "<i8"), ("nf", "<f4"), ("d", "<f4"), ("is_int", "<i4"), ("pad", "<i4")])


def _is_int(v) -> bool:
    import numbers

    return isinstance(v, numbers.Integral)


def scalar_f32(v) -> float:
    """The float32 torch's CPU kernels use for a Python scalar next to an fp32
    (or bf16 / f16: opmath float) tensor: an int converts int64 -> float
    with one round-to-nearest-even, a float double -> float."""
    if _is_int(v):
        return float(torch.tensor(int(v), dtype=torch.int64).to(torch.float32).item())
    return float(np.float32(float(v)))


def muldiv_weights(dtype: torch.dtype, pairs: Sequence, device: torch.device) -> torch.Tensor:
    """fedagg_wsum_muldiv's K weight records for (n_i, N) pairs, uploaded as
    bytes: {fl32(n_i), fl32(N)} for fp32 / bf16 / f16 rows, doubles for f64,
    {n_i, fl32(n_i), fl32(N), is_int} for int64 rows (include/fedagg.h)."""
    K = len(pairs)
    if dtype == torch.float64:
        rec = np.zeros(K, dtype=_MULDIV_D)
        rec["n"] = [float(n) for n, _ in pairs]
        rec["d"] = [float(d) for _, d in pairs]
    elif dtype == torch.int64:
        rec = np.zeros(K, dtype=_MULDIV_I)
        rec["is_int"] = [1 if _is_int(n) else 0 for n, _ in pairs]
        rec["n"] = [int(n) if _is_int(n) else 0 for n, _ in pairs]
        rec["nf"] = [scalar_f32(n) for n, _ in pairs]
        rec["d"] = [scalar_f32(d) for _, d in pairs]
    else:
        rec = np.zeros(K, dtype=_MULDIV_F)
        rec["n"] = [scalar_f32(n) for n, _ in pairs]
        rec["d"] = [scalar_f32(d) for _, d in pairs]
    raw = np.frombuffer(rec.tobytes(), dtype=np.uint8)
    host = torch.from_numpy(raw.copy())
    if _cuda_ok():
        host = host.pin_memory()
    return host.to(device, non_blocking=True)


def muldiv_ptrs(dtype: torch.dtype, d_ptrs: torch.Tensor, pairs: Sequence, K: int, N: int, out: torch.Tensor,
                aligned: bool) -> torch.Tensor:
    """fedagg_wsum_muldiv: out = Σ_i fl(fl(p_i·n_i)/N) over a device pointer
    table (the MPI simulation's term order).  Returns the uploaded weight
    records (keep them alive until the launch has run)."""
    _require_cuda(out, "muldiv")
    if N == 0:
        return None
    if dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64):
        raise TypeError(f"muldiv: unsupported dtype {dtype}")
    want = torch.float32 if dtype == torch.int64 else dtype
    if out.dtype != want:
        raise TypeError(f"muldiv: {dtype} rows produce {want}")
    w = muldiv_weights(dtype, pairs, out.device)
    flags = nat.FEDAGG_ALIGNED16 if aligned and (out.data_ptr() & 15) == 0 else 0
    nat.check(nat.lib().fedagg_wsum_muldiv(_DT_CODE[dtype], d_ptrs.data_ptr(), w.data_ptr(), K, N, out.data_ptr(),
                                           flags, nat.stream_handle()), f"muldiv[{dtype}]")
    return w


def sum_ptrs(dtype: torch.dtype, d_ptrs: torch.Tensor, K: int, N: int, out: torch.Tensor, aligned: bool) -> None:
    """Unweighted sequential sum (FedAvg_seq / FedDyn)."""
    _require_cuda(out, "sum")
    if N == 0:
        return
    if dtype not in _DT_CODE:
        raise TypeError(f"sum: unsupported dtype {dtype}")
    flags = nat.FEDAGG_ALIGNED16 if aligned and (out.data_ptr() & 15) == 0 else 0
    nat.check(nat.lib().fedagg_sum(_DT_CODE[dtype], d_ptrs.data_ptr(), K, N, out.data_ptr(), flags,
                                   nat.stream_handle()), f"sum[{dtype}]")


def wsum_tensors(tensors: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
                 acc_mode: int = ACC_REFERENCE) -> None:
    """Weighted sum of K contiguous same-shape device tensors into out."""
    dev = out.device
    ptrs = [t.data_ptr() for t in tensors]
    d_ptrs = upload_i64(ptrs, dev)
    dtype = tensors[0].dtype
    d_w = upload_f64(weights, dev) if dtype == torch.float64 else upload_f32(weights, dev)
    wsum_ptrs(dtype, d_ptrs, d_w, len(tensors), tensors[0].numel(), out, aligned16(ptrs), acc_mode)


_MULTI_DT = {torch.float32: nat.DT_F32, torch.bfloat16: nat.DT_BF16, torch.float16: nat.DT_F16,
             torch.int64: nat.DT_I64}
MULTI_DTYPES = tuple(_MULTI_DT)


def weights_as_i64(weights: Sequence[float]) -> np.ndarray:
    """fp32 weights (RNE from the Python floats, as torch.tensor rounds them)
    packed two per int64 slot, zero-padded to an even count: the tail of a
    pointer table upload, read by the kernel as K floats."""
    wf = np.asarray([float(v) for v in weights], dtype=np.float32)
    if wf.size % 2:
        wf = np.append(wf, np.float32(0.0))
    return wf.view(np.int64)


class DevPtr:
    """A device address inside a tensor (kept alive here): data_ptr() only."""

    def __init__(self, owner: torch.Tensor, ptr: int):
        self.owner = owner
        self.ptr = ptr

    def data_ptr(self) -> int:
        return self.ptr


class MultiPlan:
    """Segment table for the one-launch multi-tensor kernel (fedagg_wsum_multi):
    T keys of one dtype, each with K client pointers.  int64 keys produce
    float32 outputs (the reference's int64 * float promotion)."""

    def __init__(self, numels: Sequence[int], dtype: torch.dtype = torch.float32, acc_mode: int = 0):
        if dtype not in _MULTI_DT:
            raise TypeError(f"MultiPlan: unsupported dtype {dtype}")
        lib = nat.lib()
        self.dt = _MULTI_DT[dtype]
        self.acc_mode = int(acc_mode)
        self.numels = [int(n) for n in numels]
        begin = [0]
        for n in self.numels:
            nb = lib.fedagg_multi_blocks(self.dt, n)
            if nb < 0:
                raise ValueError("bad numel")
            begin.append(begin[-1] + nb)
        self.block_begin = begin
        self.total_blocks = begin[-1]
        self._meta = {}

    def launch(self, src_ptrs, out_ptrs: List[int], d_w, K: int, device: torch.device,
               weights: "Sequence[float] | None" = None, on_uploaded=None) -> list:
        """src_ptrs is the flattened [T][K] table (a list of ints, or an int64
        numpy array / bytes as the native dict walker produces it).  Returns
        the device tables, which must stay referenced until the launch has
        been enqueued.

        d_w None: the fp32 weights ride at the end of the pointer table's
        upload (one H2D instead of two), and the returned list ends with a
        DevPtr to them for later launches.  on_uploaded() is called after the
        upload is enqueued and before the kernel is."""
        T = len(self.numels)
        if isinstance(src_ptrs, (bytes, bytearray)):
            src_ptrs = np.frombuffer(src_ptrs, dtype=np.int64)
        if isinstance(out_ptrs, (bytes, bytearray)):
            out_ptrs = np.frombuffer(out_ptrs, dtype=np.int64)
        if len(src_ptrs) != T * K or len(out_ptrs) != T:
            raise ValueError("MultiPlan.launch: table sizes do not match the plan")
        # numels and block starts: uploaded once per device and stream (the
        # upload is ordered on that stream before every later launch on it)
        st = nat.stream_handle()
        d_meta = self._meta.get((device, st))
        if d_meta is None:
            d_meta = self._meta[(device, st)] = upload_i64(self.numels + self.block_begin, device)
        tail = []
        if d_w is None:
            if weights is None or len(weights) != K:
                raise ValueError("MultiPlan.launch: K weights needed when d_w is None")
            tail = [weights_as_i64(weights)]
        if tail or isinstance(src_ptrs, np.ndarray) or isinstance(out_ptrs, np.ndarray):
            tab = np.concatenate([np.asarray(src_ptrs, dtype=np.int64), np.asarray(out_ptrs, dtype=np.int64)] + tail)
        else:
            tab = list(src_ptrs) + list(out_ptrs)
        d_tab = upload_i64(tab, device)
        ret = [d_meta, d_tab]
        if d_w is None:
            d_w = DevPtr(d_tab, d_tab.data_ptr() + 8 * (T * K + T))
            ret.append(d_w)
        if on_uploaded is not None:
            on_uploaded()
        nat.check(nat.lib().fedagg_wsum_multi(self.dt, self.acc_mode, d_tab.data_ptr(), d_tab.data_ptr() + 8 * T * K,
                                              d_meta.data_ptr(), d_meta.data_ptr() + 8 * T, T, d_w.data_ptr(), K,
                                              self.total_blocks, st), "wsum_multi")
        return ret


class MultiF32Plan(MultiPlan):
    """fp32 MultiPlan (kept for callers of the fp32-only entry point)."""

    def __init__(self, numels: Sequence[int]):
        super().__init__(numels, torch.float32)


def fedopt_sgd(param: torch.Tensor, mom: torch.Tensor | None, avg: torch.Tensor, lr: float, momentum: float,
               first_step: bool) -> None:
    """Fused server SGD(+momentum) step on flat fp32 device tensors, in place."""
    _require_cuda(param, "fedopt_sgd")
    if param.dtype != torch.float32 or avg.dtype != torch.float32:
        raise TypeError("fedopt_sgd: fp32 only")
    nat.check(nat.lib().fedagg_fedopt_sgd_f32(param.data_ptr(), mom.data_ptr() if mom is not None else None,
                                              avg.data_ptr(), param.numel(), float(lr), float(momentum),
                                              int(first_step), nat.stream_handle()), "fedopt_sgd_f32")


def wsum_fedopt_sgd(d_ptrs: torch.Tensor, d_w: torch.Tensor, K: int, N: int, param: torch.Tensor,
                    mom: torch.Tensor | None, lr: float, momentum: float, first_step: bool, aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server SGD step: param (flat,
    N elements) goes from p_old to p_new in place, mom is the momentum buffer."""
    _require_cuda(param, "wsum_fedopt_sgd")
    ok = aligned and (param.data_ptr() & 15) == 0 and (mom is None or (mom.data_ptr() & 15) == 0)
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_sgd_f32(
        d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), mom.data_ptr() if mom is not None else None,
        float(lr), float(momentum), int(first_step), flags, nat.stream_handle()), "wsum_fedopt_sgd_f32")


def adam_scalars(lr: float, beta1: float, beta2: float, eps: float, step: int) -> "ctypes.Array":
    """The six fp32 scalars of one torch Adam step (fedagg_adam_scalars), as a
    host array to pass to wsum_fedopt_adam."""
    out = (ctypes.c_float * 6)()
    nat.check(nat.lib().fedagg_adam_scalars(float(lr), float(beta1), float(beta2), float(eps), int(step),
                                            ctypes.addressof(out)), "adam_scalars")
    return out


def wsum_fedopt_adam(d_ptrs: torch.Tensor, d_w: torch.Tensor, K: int, N: int, param: torch.Tensor,
                     exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, scalars: "ctypes.Array", first_step: bool,
                     aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server Adam step: param, exp_avg
    and exp_avg_sq (flat, N elements each) are updated in place."""
    _require_cuda(param, "wsum_fedopt_adam")
    ok = aligned and all((t.data_ptr() & 15) == 0 for t in (param, exp_avg, exp_avg_sq))
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_adam_f32(
        d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
        ctypes.addressof(scalars), int(first_step), flags, nat.stream_handle()), "wsum_fedopt_adam_f32")


def wsum_fedopt_adagrad(d_ptrs: torch.Tensor, d_w, K: int, N: int, param: torch.Tensor, state_sum: torch.Tensor,
                        clr: float, eps: float, aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server Adagrad step: param and
    state_sum (flat, N elements each) are updated in place."""
    _require_cuda(param, "wsum_fedopt_adagrad")
    ok = aligned and all((t.data_ptr() & 15) == 0 for t in (param, state_sum))
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_adagrad_f32(
        d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), state_sum.data_ptr(), float(clr), float(eps),
        flags, nat.stream_handle()), "wsum_fedopt_adagrad_f32")


def wsum_fedopt_adamw(d_ptrs: torch.Tensor, d_w, K: int, N: int, param: torch.Tensor, exp_avg: torch.Tensor,
                      exp_avg_sq: torch.Tensor, scalars: "ctypes.Array", decay: float, first_step: bool,
                      aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server AdamW step (decay =
    1 - lr * weight_decay, rounded to fp32 by ctypes as torch rounds it)."""
    _require_cuda(param, "wsum_fedopt_adamw")
    ok = aligned and all((t.data_ptr() & 15) == 0 for t in (param, exp_avg, exp_avg_sq))
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_adamw_f32(
        d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
        ctypes.addressof(scalars), float(decay), int(first_step), flags, nat.stream_handle()),
        "wsum_fedopt_adamw_f32")


def wsum_fedopt_rmsprop(d_ptrs: torch.Tensor, d_w, K: int, N: int, param: torch.Tensor, square_avg: torch.Tensor,
                        lr: float, alpha: float, eps: float, aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server RMSprop step."""
    _require_cuda(param, "wsum_fedopt_rmsprop")
    ok = aligned and all((t.data_ptr() & 15) == 0 for t in (param, square_avg))
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_rmsprop_f32(
        d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), square_avg.data_ptr(), float(lr), float(alpha),
        float(eps), flags, nat.stream_handle()), "wsum_fedopt_rmsprop_f32")


def optrepo_scalars(opt: str, lr: float, step: int, carry: "ctypes.Array") -> "ctypes.Array":
    """The nine fp32 scalars of one step of an OptRepo optimizer
    (fedagg_optrepo_scalars; `carry` is its fp32 scalar state, two floats,
    updated in place: NAdam's mu_product, ASGD's eta and mu)."""
    out = (ctypes.c_float * 9)()
    nat.check(nat.lib().fedagg_optrepo_scalars(nat.OPT_CODES[opt], float(lr), int(step), ctypes.addressof(carry),
                                               ctypes.addressof(out)), "optrepo_scalars")
    return out


def wsum_fedopt_optrepo(opt: str, d_ptrs: torch.Tensor, d_w, K: int, N: int, param: torch.Tensor,
                        state0: torch.Tensor, state1: Optional[torch.Tensor], scalars: "ctypes.Array",
                        aligned: bool) -> None:
    """FedAvg of K fp32 sources fused with the server step of an OptRepo
    optimizer (adamax / nadam / radam / adadelta / asgd / rprop): param and
    the state buffers (flat, N elements each) are updated in place."""
    _require_cuda(param, "wsum_fedopt_optrepo")
    ts = [t for t in (param, state0, state1) if t is not None]
    ok = aligned and all((t.data_ptr() & 15) == 0 for t in ts)
    flags = (nat.FEDAGG_ALIGNED16 if ok else 0) | (nat.FEDAGG_HOST_WEIGHTS if isinstance(d_w, HostWeights) else 0)
    nat.check(nat.lib().fedagg_wsum_fedopt_optrepo_f32(
        nat.OPT_CODES[opt], d_ptrs.data_ptr(), d_w.data_ptr(), K, N, param.data_ptr(), state0.data_ptr(),
        state1.data_ptr() if state1 is not None else None, ctypes.addressof(scalars), flags, nat.stream_handle()),
        f"wsum_fedopt_optrepo_f32 ({opt})")


def round_f32(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """fp32 -> bf16/f16 (RNE) on the device, in libfedagg (fedagg_round_f32)."""
    _require_cuda(x, "round_f32")
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    nat.check(nat.lib().fedagg_round_f32(_DT_CODE[dtype], x.data_ptr(), x.numel(), out.data_ptr(),
                                         nat.stream_handle()), "round_f32")
    return out
