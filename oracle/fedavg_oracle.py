"""numpy restatement of FedML's torch_aggregator — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP path.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it; the
product package fedml_amd/ never does.

It restates, branch by branch, python/fedml/ml/aggregator/agg_operator.py:
  FedMLAggOperator.agg            :10-30   (Σ n_i, tuple arity per optimizer)
  torch_aggregator  FedAvg        :35-44
                    FedProx       :45-54   (identical arithmetic)
                    FedAvg_seq    :55-63   (unweighted, aliases client 0)
                    FedOpt/FedNova :64-67  (`pass` -> UnboundLocalError)
                    FedDyn        :68-77   (unweighted, aliases client 0)
                    SCAFFOLD      :100-118 (overwrites with the last client)
                    Mime          :119-133
and the FedOpt server step of simulation/mpi/fedopt/FedOptAggregator.py:81-130
(SGD) and of sp/fedopt/fedopt_api.py:121-130 (Adam, Adagrad), and the MPI
simulation's FedAvg term order (simulation/mpi/fedavg/FedAVGAggregator.py:
99-116, mpi_fedavg).

Inputs and outputs are CPU torch tensors (the reference's own currency); all
arithmetic is numpy in the tensor's opmath type with one IEEE rounding per
operation, exactly as torch's CPU kernels round (the conventions are stated in
oracle/fedavg_oracle.c).  Pinned against golden vectors produced by the
reference itself: tests/golden/ (see tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from collections import OrderedDict
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
_CLIB = os.path.join(HERE, "_build", "liboracle.so")

_INT_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)


# --------------------------------------------------------------------------
# bf16 / dtype helpers


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """c10::BFloat16 round-to-nearest-even; NaN -> 0x7FC0."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[np.isnan(x)] = 0x7FC0
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.ascontiguousarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def _rbf(x: np.ndarray) -> np.ndarray:
    return bf16_bits_to_f32(f32_to_bf16_bits(x))


def _rf16(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).astype(np.float32)


def to_np(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()


def from_np(a: np.ndarray, dtype: torch.dtype, shape) -> torch.Tensor:
    if dtype == torch.bfloat16:
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).reshape(shape)
    return torch.from_numpy(np.ascontiguousarray(a)).reshape(shape).to(dtype)


def weight_f32(n_i, total) -> np.float32:
    """agg_operator.py:39 `w = local_sample_number / training_num` (Python
    float64 division; ZeroDivisionError when Σn == 0), then torch rounds the
    scalar to the float32 opmath type."""
    return np.float32(n_i / total)


# --------------------------------------------------------------------------
# Per-tensor chains


def wsum(tensors: Sequence[torch.Tensor], ws: Sequence[float]) -> torch.Tensor:
    """One state-dict key: avg = p_0*w_0 ; avg += p_i*w_i (agg_operator.py:40-44).

    ws are the Python-float weights n_i / Σn.  Output dtype follows torch's
    promotion of `tensor * python_float`: float types keep their dtype,
    integer/bool tensors become float32."""
    dt = tensors[0].dtype
    shape = tensors[0].shape
    if dt == torch.float32 or dt in _INT_DTYPES:
        w32 = [np.float32(w) for w in ws]
        acc = to_np(tensors[0]).astype(np.float32) * w32[0]
        for t, w in zip(tensors[1:], w32[1:]):
            acc = acc + to_np(t).astype(np.float32) * w
        return from_np(acc.astype(np.float32), torch.float32, shape)
    if dt == torch.float64:
        acc = to_np(tensors[0]) * np.float64(ws[0])
        for t, w in zip(tensors[1:], ws[1:]):
            acc = acc + to_np(t) * np.float64(w)
        return from_np(acc, torch.float64, shape)
    if dt in (torch.bfloat16, torch.float16):
        r = _rbf if dt == torch.bfloat16 else _rf16
        conv = bf16_bits_to_f32 if dt == torch.bfloat16 else (lambda a: a.astype(np.float32))
        w32 = [np.float32(w) for w in ws]
        acc = r(conv(to_np(tensors[0])) * w32[0])
        for t, w in zip(tensors[1:], w32[1:]):
            acc = r(acc + r(conv(to_np(t)) * w))
        if dt == torch.bfloat16:
            return from_np(f32_to_bf16_bits(acc), torch.bfloat16, shape)
        return from_np(acc.astype(np.float16), torch.float16, shape)
    raise TypeError(f"oracle: unsupported dtype {dt}")


def wsum_acc32(tensors: Sequence[torch.Tensor], ws: Sequence[float]) -> torch.Tensor:
    """fedml_amd's `fedagg_low_precision_acc="fp32"` mode for bf16/f16 keys
    (not a reference behaviour; the definition its kernels are checked
    against): acc = fl32(x_0 * fl32(w_0)); acc = fl32(acc + fl32(x_i * fl32(w_i)))
    in fp32, one RNE to the key's dtype at the end."""
    dt = tensors[0].dtype
    conv = bf16_bits_to_f32 if dt == torch.bfloat16 else (lambda a: a.astype(np.float32))
    w32 = [np.float32(w) for w in ws]
    acc = conv(to_np(tensors[0])) * w32[0]
    for t, w in zip(tensors[1:], w32[1:]):
        acc = acc + conv(to_np(t)) * w
    if dt == torch.bfloat16:
        return from_np(f32_to_bf16_bits(acc), torch.bfloat16, tensors[0].shape)
    return from_np(acc.astype(np.float16), torch.float16, tensors[0].shape)


def seqsum(tensors: Sequence[torch.Tensor]) -> np.ndarray:
    """avg = p_0 ; avg += p_i in the source dtype (agg_operator.py:58-63)."""
    dt = tensors[0].dtype
    if dt == torch.bfloat16:
        acc = bf16_bits_to_f32(to_np(tensors[0]))
        for t in tensors[1:]:
            acc = _rbf(acc + bf16_bits_to_f32(to_np(t)))
        return f32_to_bf16_bits(acc)
    if dt == torch.float16:
        acc = to_np(tensors[0]).astype(np.float32)
        for t in tensors[1:]:
            acc = _rf16(acc + to_np(t).astype(np.float32))
        return acc.astype(np.float16)
    acc = to_np(tensors[0])
    for t in tensors[1:]:
        with np.errstate(over="ignore"):
            acc = acc + to_np(t)  # integer adds wrap like torch's
    return acc.astype(to_np(tensors[0]).dtype)


# --------------------------------------------------------------------------
# FedMLAggOperator.agg restatement


def agg(args, raw_grad_list):
    """agg_operator.py:10-30 then torch_aggregator :33-134.  Mutates the
    client-0 dicts exactly as the reference does."""
    opt = args.federated_optimizer
    training_num = 0
    if opt in ("SCAFFOLD", "Mime"):
        for item in raw_grad_list:
            local_sample_num, _, _ = item
            training_num += local_sample_num
    else:
        for item in raw_grad_list:
            local_sample_num, _ = item
            training_num += local_sample_num
    return torch_aggregator(args, raw_grad_list, training_num)


def scale(t: torch.Tensor, w: float) -> torch.Tensor:
    """torch's `t * w` for a Python-float w, one rounding in the opmath type:
    float types keep their dtype, integer / bool tensors become float32
    (agg_operator.py:41,44 `local_model_params[k] * w`)."""
    dt = t.dtype
    if dt == torch.float32 or dt in _INT_DTYPES:
        return from_np((to_np(t).astype(np.float32) * np.float32(w)).astype(np.float32), torch.float32, t.shape)
    if dt == torch.float64:
        return from_np(to_np(t) * np.float64(w), torch.float64, t.shape)
    if dt == torch.bfloat16:
        return from_np(f32_to_bf16_bits(bf16_bits_to_f32(to_np(t)) * np.float32(w)), torch.bfloat16, t.shape)
    if dt == torch.float16:
        return from_np((to_np(t).astype(np.float32) * np.float32(w)).astype(np.float16), torch.float16, t.shape)
    raise TypeError(f"oracle: unsupported dtype {dt}")


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """torch's `a += b` for same-dtype tensors (float32 when a promoted
    integer key meets a float32 one): one rounding in the dtype; integer adds
    wrap."""
    dt = a.dtype
    if dt == torch.bfloat16:
        return from_np(f32_to_bf16_bits(bf16_bits_to_f32(to_np(a)) + bf16_bits_to_f32(to_np(b))), dt, a.shape)
    if dt == torch.float16:
        return from_np((to_np(a).astype(np.float32) + to_np(b).astype(np.float32)).astype(np.float16), dt, a.shape)
    if dt == torch.float32:
        return from_np(to_np(a) + to_np(b).astype(np.float32), dt, a.shape)
    with np.errstate(over="ignore"):
        return from_np((to_np(a) + to_np(b)).astype(to_np(a).dtype), dt, a.shape)


def _set_inplace(t: torch.Tensor, v: torch.Tensor) -> None:
    """`t += x` keeps t's storage: write v's bits into t."""
    if t.dtype == torch.bfloat16:
        t.view(torch.int16).copy_(v.view(torch.int16).reshape(t.shape))
    else:
        t.copy_(v.reshape(t.shape))


def torch_aggregator(args, raw_grad_list, training_num):
    """agg_operator.py:33-134 step by step: every client's tensors are looked
    up in its dict at the moment the reference's loop reads them, so a dict
    listed twice reads the running accumulator exactly as the reference does
    (the accumulator IS client 0's dict entry; FedAvg_seq / FedDyn and
    SCAFFOLD's control variates add into client 0's own tensors in place)."""
    opt = args.federated_optimizer
    K = len(raw_grad_list)
    if opt in ("FedAvg", "FedProx"):
        avg_params = raw_grad_list[0][1]
        for k in list(avg_params.keys()):
            for i in range(K):
                local_sample_number, local_model_params = raw_grad_list[i]
                w = local_sample_number / training_num
                x = scale(local_model_params[k], w)
                avg_params[k] = x if i == 0 else add(avg_params[k], x)
        return avg_params
    if opt in ("FedAvg_seq", "FedDyn"):
        avg_params = raw_grad_list[0][1]
        for k in list(avg_params.keys()):
            for i in range(K):
                local_model_params = raw_grad_list[i][1]
                if i == 0:
                    avg_params[k] = local_model_params[k]  # client 0's own tensor, summed into in place
                else:
                    _set_inplace(avg_params[k], add(avg_params[k], local_model_params[k]))
        return avg_params
    if opt == "SCAFFOLD":
        total_weights_delta, total_c_delta_para = raw_grad_list[0][1], raw_grad_list[0][2]
        w_c = 1 / args.client_num_in_total
        for k in list(total_weights_delta.keys()):
            for i in range(K):
                local_sample_number, weights_delta, c_delta_para = raw_grad_list[i]
                w = local_sample_number / training_num
                if i == 0:
                    total_weights_delta[k] = scale(weights_delta[k], w)
                    total_c_delta_para[k] = c_delta_para[k]  # bound, then `+=` in place (:110,113)
                else:
                    total_weights_delta[k] = add(total_weights_delta[k], scale(weights_delta[k], w))
                    _set_inplace(total_c_delta_para[k], add(total_c_delta_para[k], c_delta_para[k]))
            # :116-117 overwrite both with the LAST client's entries (which are
            # the running sums themselves when that client's dicts are client 0's)
            total_weights_delta[k] = weights_delta[k]
            total_c_delta_para[k] = scale(c_delta_para[k], w_c)
        return (total_weights_delta, total_c_delta_para)
    if opt == "Mime":
        avg_params, avg_local_grad = raw_grad_list[0][1], raw_grad_list[0][2]
        assert args.client_num_per_round == K
        for k in list(avg_params.keys()):
            for i in range(K):
                local_sample_number, local_model_params, local_grad = raw_grad_list[i]
                w = local_sample_number / training_num
                if i == 0:
                    avg_params[k] = scale(local_model_params[k], w)
                    avg_local_grad[k] = scale(local_grad[k], w)
                else:
                    avg_params[k] = add(avg_params[k], scale(local_model_params[k], w))
                    avg_local_grad[k] = add(avg_local_grad[k], scale(local_grad[k], w))
        return (avg_params, avg_local_grad)
    # FedOpt, FedNova (`pass`) and unknown names leave avg_params unbound.
    raise UnboundLocalError("local variable 'avg_params' referenced before assignment")


# --------------------------------------------------------------------------
# MPI simulation FedAvg (simulation/mpi/fedavg/FedAVGAggregator.py:99-116)


def _f32_scalar(v) -> np.float32:
    """A Python scalar as torch's CPU kernels take it next to an fp32 / bf16 /
    f16 tensor: int -> int64 -> float (one RNE), float -> double -> float."""
    import numbers

    if isinstance(v, numbers.Integral):
        return np.float32(torch.tensor(int(v), dtype=torch.int64).to(torch.float32).item())
    return np.float32(float(v))


def mul_scalar(t: torch.Tensor, n) -> torch.Tensor:
    """torch's `t * n` for a Python scalar n (FedAVGAggregator.py:108,112):
    int64 / bool tensors times an int stay int64 (two's-complement wrap),
    times a float promote to float32; float tensors round once in their
    opmath type (f16: the fp32 product, then f16)."""
    import numbers

    dt = t.dtype
    if dt in (torch.int64, torch.bool) and isinstance(n, numbers.Integral):
        with np.errstate(over="ignore"):
            prod = np.asarray(to_np(t).astype(np.int64) * np.int64(int(n)), dtype=np.int64)
            return torch.from_numpy(prod.copy()).reshape(t.shape)
    if dt == torch.float64:
        return from_np(to_np(t) * np.float64(n), dt, t.shape)
    if dt == torch.bfloat16:
        return from_np(f32_to_bf16_bits(bf16_bits_to_f32(to_np(t)) * _f32_scalar(n)), dt, t.shape)
    if dt == torch.float16:
        return from_np((to_np(t).astype(np.float32) * _f32_scalar(n)).astype(np.float16), dt, t.shape)
    if dt == torch.float32 or dt in (torch.int64, torch.bool):
        return from_np((to_np(t).astype(np.float32) * _f32_scalar(n)).astype(np.float32), torch.float32, t.shape)
    raise TypeError(f"oracle: unsupported dtype {dt}")


def div_scalar(t: torch.Tensor, d) -> torch.Tensor:
    """torch's true division `t / d` by a Python scalar: integer tensors
    promote to float32 (fl32(v) / fl32(d)), float tensors divide by the
    scalar rounded to their opmath type."""
    dt = t.dtype
    with np.errstate(divide="ignore", invalid="ignore"):
        if dt == torch.float64:
            return from_np(to_np(t) / np.float64(d), dt, t.shape)
        if dt == torch.bfloat16:
            return from_np(f32_to_bf16_bits(bf16_bits_to_f32(to_np(t)) / _f32_scalar(d)), dt, t.shape)
        if dt == torch.float16:
            return from_np((to_np(t).astype(np.float32) / _f32_scalar(d)).astype(np.float16), dt, t.shape)
        return from_np((to_np(t).astype(np.float32) / _f32_scalar(d)).astype(np.float32), torch.float32, t.shape)


def mpi_fedavg(model_list):
    """FedAVGAggregator._fedavg_aggregation_ (:99-116) step by step: each term
    `local_model_params[k] * local_sample_number / training_num` left to right,
    accumulated into client 0's dict (live lookups: a dict listed again reads
    the running sum)."""
    training_num = 0
    for i in range(len(model_list)):
        local_sample_number, local_model_params = model_list[i]
        training_num += local_sample_number
    (num0, averaged_params) = model_list[0]
    for k in list(averaged_params.keys()):
        for i in range(len(model_list)):
            local_sample_number, local_model_params = model_list[i]
            x = div_scalar(mul_scalar(local_model_params[k], local_sample_number), training_num)
            averaged_params[k] = x if i == 0 else add(averaged_params[k], x)
    return averaged_params


# --------------------------------------------------------------------------
# C oracle (exact fmaf for the FedOpt step; scalar cross-check of wsum)


def build_c(force: bool = False) -> str:
    src = os.path.join(HERE, "fedavg_oracle.c")
    if force or not os.path.exists(_CLIB) or os.path.getmtime(src) > os.path.getmtime(_CLIB):
        subprocess.run(["make", "-s", "-C", HERE, "_build/liboracle.so"], check=True)
    return _CLIB


_clib = None


def clib() -> ctypes.CDLL:
    global _clib
    if _clib is None:
        lib = ctypes.CDLL(build_c())
        P, I, L, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
        for name, args in {
            "oracle_wsum_f32": [P, P, I, L, P],
            "oracle_wsum_bf16": [P, P, I, L, P],
            "oracle_wsum_i64_f32": [P, P, I, L, P],
            "oracle_wsum_f64": [P, P, I, L, P],
            "oracle_sum_f32": [P, I, L, P],
            "oracle_sum_bf16": [P, I, L, P],
            "oracle_sum_i64": [P, I, L, P],
            "oracle_fedopt_sgd_f32": [P, P, P, L, F, F, I],
            "oracle_adam_moments_f32": [P, P, P, P, L, F, F, F],
            "oracle_adagrad_sum_f32": [P, P, P, L],
            "oracle_fma_f32": [P, P, P, P, L],
        }.items():
            fn = getattr(lib, name)
            fn.restype = None
            fn.argtypes = args
        _clib = lib
    return _clib


def c_wsum(arrays: List[np.ndarray], ws: Sequence[float]) -> np.ndarray:
    """Weighted sum through the C oracle; arrays are 1-D numpy arrays of one
    dtype (float32, uint16 = bf16 bits, int64, float64)."""
    lib = clib()
    K = len(arrays)
    arrays = [np.ascontiguousarray(a) for a in arrays]
    N = arrays[0].size
    ptrs = (ctypes.c_void_p * K)(*[a.ctypes.data for a in arrays])
    dt = arrays[0].dtype
    if dt == np.float64:
        w = np.asarray(ws, dtype=np.float64)
        out = np.empty(N, np.float64)
        lib.oracle_wsum_f64(ptrs, w.ctypes.data, K, N, out.ctypes.data)
        return out
    w = np.asarray([np.float32(x) for x in ws], dtype=np.float32)
    if dt == np.float32:
        out = np.empty(N, np.float32)
        lib.oracle_wsum_f32(ptrs, w.ctypes.data, K, N, out.ctypes.data)
    elif dt == np.uint16:
        out = np.empty(N, np.uint16)
        lib.oracle_wsum_bf16(ptrs, w.ctypes.data, K, N, out.ctypes.data)
    elif dt == np.int64:
        out = np.empty(N, np.float32)
        lib.oracle_wsum_i64_f32(ptrs, w.ctypes.data, K, N, out.ctypes.data)
    else:
        raise TypeError(dt)
    return out


def fedopt_sgd(p_old: np.ndarray, avg: np.ndarray, buf: np.ndarray | None, lr: float, momentum: float,
               first: bool) -> Tuple[np.ndarray, np.ndarray | None]:
    """One server SGD step on one named parameter (FedOptAggregator.py:104-125)."""
    p = np.ascontiguousarray(p_old, dtype=np.float32).copy()
    a = np.ascontiguousarray(avg, dtype=np.float32)
    b = np.zeros_like(p) if buf is None else np.ascontiguousarray(buf, dtype=np.float32).copy()
    clib().oracle_fedopt_sgd_f32(p.ctypes.data, b.ctypes.data, a.ctypes.data, p.size, float(lr),
                                 float(momentum), int(first))
    return p, (b if momentum != 0 else None)


def adam_scalars(lr: float, beta1: float, beta2: float, eps: float, step: int) -> Tuple[float, ...]:
    """The double-precision scalars of torch's _single_tensor_adam for 1-based
    `step`, each as the fp32 value the CPU kernel receives: (lerp weight, beta2,
    addcmul value, bias_correction2 ** 0.5, eps, -step_size)."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    vals = (1 - beta1, beta2, 1 - beta2, bc2 ** 0.5, eps, -(lr / bc1))
    return tuple(float(np.float32(v)) for v in vals)


def fedopt_adam(p_old: np.ndarray, avg: np.ndarray, m: np.ndarray | None, v: np.ndarray | None, lr: float,
                step: int, betas=(0.9, 0.999), eps: float = 1e-8, sqrt: str = "torch", weight_decay: float = 0.0
                ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """One server Adam step on one named parameter (sp/fedopt/fedopt_api.py:121-130,
    grad = p_old - avg as _set_model_global_grads :155-160).  Returns (p, m, v).

    sqrt="torch" uses torch's CPU sqrt, which is what the reference's
    exp_avg_sq.sqrt() runs (on this image an MKL VML routine that is NOT
    correctly rounded: ~0.6% of fp32 results are 1 ulp off); sqrt="ieee" uses
    the correctly rounded sqrt the GPU kernel computes.

    weight_decay != 0 is torch.optim.AdamW (Adam with decoupled weight decay):
    param.mul_(1 - lr * weight_decay) runs first, the gradient having been set
    from the unscaled parameter, so p = fl(p_old * fl32(1 - lr*wd)) + step."""
    w1, b2, c2, bc2s, epsf, nss = (np.float32(x) for x in adam_scalars(lr, betas[0], betas[1], eps, step))
    p = np.ascontiguousarray(p_old, dtype=np.float32).reshape(-1).copy()
    a = np.ascontiguousarray(avg, dtype=np.float32).reshape(-1)
    mm = np.zeros_like(p) if m is None else np.ascontiguousarray(m, dtype=np.float32).reshape(-1).copy()
    vv = np.zeros_like(p) if v is None else np.ascontiguousarray(v, dtype=np.float32).reshape(-1).copy()
    clib().oracle_adam_moments_f32(p.ctypes.data, a.ctypes.data, mm.ctypes.data, vv.ctypes.data, p.size,
                                   float(w1), float(b2), float(c2))
    if sqrt == "torch":
        s = torch.from_numpy(vv).sqrt().numpy()
    elif sqrt == "ieee":
        s = np.sqrt(vv)
    else:
        raise ValueError(sqrt)
    denom = (s / bc2s) + epsf  # (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
    if weight_decay:
        p = (p * np.float32(1 - lr * weight_decay)).astype(np.float32)  # param.mul_(1 - lr * wd)
    p = (p + (nss * mm) / denom).astype(np.float32)  # addcdiv_: self + (value * t1) / t2
    return p, mm, vv


def fedopt_adam_round(global_sd: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str], raw_grad_list,
                      lr: float, state: Dict[str, Tuple[np.ndarray, np.ndarray]], step: int,
                      sqrt: str = "torch", weight_decay: float = 0.0) -> "OrderedDict[str, torch.Tensor]":
    """One FedOptAPI round with server_optimizer="adam" (fedopt_api.py:121-130):
    FedAvg, Adam on named parameters (state carries exp_avg / exp_avg_sq across
    rounds, step is 1-based), averaged values for buffers."""
    class _A:
        federated_optimizer = "FedAvg"
    avg = agg(_A(), raw_grad_list)
    out = OrderedDict()
    for k, t_old in global_sd.items():
        if k in param_names:
            m, v = state.get(k, (None, None))
            p, m, v = fedopt_adam(to_np(t_old).ravel(), to_np(avg[k]).ravel(), m, v, lr, step, sqrt=sqrt,
                                  weight_decay=weight_decay)
            state[k] = (m, v)
            out[k] = torch.from_numpy(p).reshape(t_old.shape)
        else:
            out[k] = avg[k].to(t_old.dtype).reshape(t_old.shape)
    return out


def fedopt_adagrad(p_old: np.ndarray, avg: np.ndarray, acc: np.ndarray | None, lr: float, eps: float = 1e-10,
                   sqrt: str = "torch") -> Tuple[np.ndarray, np.ndarray]:
    """One server Adagrad step on one named parameter (torch.optim.Adagrad with
    lr only, as sp/fedopt/fedopt_api.py:78-85 builds it; lr_decay 0 so the
    step's clr is lr).  Returns (p, state_sum):
      sum = fma(g, g, sum)                     addcmul_(g, g, value=1)
      std = fl(sqrt(sum) + eps)                sqrt().add_(eps)
      p   = fl(p + fl(fl(-clr * g) / std))     addcdiv_(g, std, value=-clr), not fused
    sqrt as in fedopt_adam (torch's CPU sqrt is not correctly rounded)."""
    p = np.ascontiguousarray(p_old, dtype=np.float32).reshape(-1).copy()
    a = np.ascontiguousarray(avg, dtype=np.float32).reshape(-1)
    ss = np.zeros_like(p) if acc is None else np.ascontiguousarray(acc, dtype=np.float32).reshape(-1).copy()
    clib().oracle_adagrad_sum_f32(p.ctypes.data, a.ctypes.data, ss.ctypes.data, p.size)
    g = (p - a).astype(np.float32)
    if sqrt == "torch":
        r = torch.from_numpy(ss).sqrt().numpy()
    elif sqrt == "ieee":
        r = np.sqrt(ss)
    else:
        raise ValueError(sqrt)
    std = (r + np.float32(eps)).astype(np.float32)
    p = (p + (np.float32(-lr) * g) / std).astype(np.float32)
    return p, ss


def fedopt_adagrad_round(global_sd: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str], raw_grad_list,
                         lr: float, state: Dict[str, np.ndarray], sqrt: str = "torch"
                         ) -> "OrderedDict[str, torch.Tensor]":
    """One FedOptAPI round with server_optimizer="adagrad" (fedopt_api.py:121-130):
    FedAvg, Adagrad on named parameters (state carries state_sum across rounds),
    averaged values for buffers."""
    class _A:
        federated_optimizer = "FedAvg"
    avg = agg(_A(), raw_grad_list)
    out = OrderedDict()
    for k, t_old in global_sd.items():
        if k in param_names:
            p, state[k] = fedopt_adagrad(to_np(t_old).ravel(), to_np(avg[k]).ravel(), state.get(k), lr, sqrt=sqrt)
            out[k] = torch.from_numpy(p).reshape(t_old.shape)
        else:
            out[k] = avg[k].to(t_old.dtype).reshape(t_old.shape)
    return out


def fedopt_rmsprop(p_old: np.ndarray, avg: np.ndarray, sq: np.ndarray | None, lr: float, alpha: float = 0.99,
                   eps: float = 1e-8, sqrt: str = "torch") -> Tuple[np.ndarray, np.ndarray]:
    """One server RMSprop step on one named parameter (torch.optim.RMSprop's
    single-tensor CPU path with momentum 0, not centered, weight_decay 0, as
    FedOptAPI builds it with lr only).  Returns (p, square_avg):
      sq  = fma(fl(fl32(1-alpha) * g), g, fl(sq * fl32(alpha)))   mul_(alpha).addcmul_(g, g, value=1-alpha)
      avg = fl(sqrt(sq) + eps)                                      sqrt().add_(eps)
      p   = fl(p + fl(fl(-lr * g) / avg))                           addcdiv_(g, avg, value=-lr)
    The accumulator update is the one Adam's exp_avg_sq takes (same torch
    kernels), so the C oracle's moment routine computes it."""
    p = np.ascontiguousarray(p_old, dtype=np.float32).reshape(-1).copy()
    a = np.ascontiguousarray(avg, dtype=np.float32).reshape(-1)
    ss = np.zeros_like(p) if sq is None else np.ascontiguousarray(sq, dtype=np.float32).reshape(-1).copy()
    unused = np.zeros_like(p)
    clib().oracle_adam_moments_f32(p.ctypes.data, a.ctypes.data, unused.ctypes.data, ss.ctypes.data, p.size,
                                   0.0, float(np.float32(alpha)), float(np.float32(1 - alpha)))
    g = (p - a).astype(np.float32)
    if sqrt == "torch":
        r = torch.from_numpy(ss).sqrt().numpy()
    elif sqrt == "ieee":
        r = np.sqrt(ss)
    else:
        raise ValueError(sqrt)
    d = (r + np.float32(eps)).astype(np.float32)
    p = (p + (np.float32(-lr) * g) / d).astype(np.float32)
    return p, ss


def fedopt_rmsprop_round(global_sd: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str], raw_grad_list,
                         lr: float, state: Dict[str, np.ndarray], sqrt: str = "torch"
                         ) -> "OrderedDict[str, torch.Tensor]":
    """One FedOptAPI round with server_optimizer="rmsprop" (fedopt_api.py:121-130)."""
    class _A:
        federated_optimizer = "FedAvg"
    avg = agg(_A(), raw_grad_list)
    out = OrderedDict()
    for k, t_old in global_sd.items():
        if k in param_names:
            p, state[k] = fedopt_rmsprop(to_np(t_old).ravel(), to_np(avg[k]).ravel(), state.get(k), lr, sqrt=sqrt)
            out[k] = torch.from_numpy(p).reshape(t_old.shape)
        else:
            out[k] = avg[k].to(t_old.dtype).reshape(t_old.shape)
    return out


# The other elementwise optimizers OptRepo can name (sp/fedopt/optrepo.py:10,
# the direct subclasses of torch.optim.Optimizer), each as FedOptAPI builds it
# (lr only, torch defaults; fedopt_api.py:78-85) and steps it on grad =
# p_old - avg (_set_model_global_grads :155-160), following torch 2.10's
# single-tensor CPU paths op by op (torch/optim/{adamax,nadam,radam,adadelta,
# asgd,rprop}.py, _single_tensor_*).  Every torch op is one IEEE rounding; the
# fused ones are fmaf through the C oracle:
#   lerp_(g, w)             fma(w, g - m, m) for w < 0.5, else fma(w - 1, g - m, g)
#   mul_(b).addcmul_(x, x, value=c)   fma(fl(c * x), x, fl(s * b))
#   add_(x, alpha=a)        fma(x, a, s)
#   addcdiv_(x, d, value=c) s + fl(fl(c * x) / d)   (not fused)
#   tensor / python float   divides by the float rounded to fp32
#   python float / tensor   Tensor.__rtruediv__: fl(fl(1 / t) * fl32(float))
# Scalars (bias corrections, NAdam's mu products, ASGD's eta) are computed in
# double as torch computes them, and rounded to fp32 where a kernel takes them;
# NAdam's mu_product and ASGD's eta / mu are fp32 state tensors.
# sqrt: "torch" (torch's CPU sqrt, an MKL routine on this image, not
# correctly rounded) or "ieee" (what the GPU computes), as for Adam.

OPTREPO_STATE = {"adamax": ("exp_avg", "exp_inf"), "nadam": ("exp_avg", "exp_avg_sq"),
                 "radam": ("exp_avg", "exp_avg_sq"), "adadelta": ("square_avg", "acc_delta"),
                 "asgd": ("ax",), "rprop": ("prev", "step_size")}


def _fma(a, b, c) -> np.ndarray:
    n = max(np.size(a), np.size(b), np.size(c))
    a, b, c = (np.ascontiguousarray(np.broadcast_to(np.float32(x) if np.ndim(x) == 0 else x, (n,)),
                                    dtype=np.float32) for x in (a, b, c))
    out = np.empty(n, np.float32)
    clib().oracle_fma_f32(a.ctypes.data, b.ctypes.data, c.ctypes.data, out.ctypes.data, n)
    return out


def _sqrt(x: np.ndarray, sqrt: str) -> np.ndarray:
    if sqrt == "torch":
        return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).sqrt().numpy()
    if sqrt == "ieee":
        return np.sqrt(x).astype(np.float32)
    raise ValueError(sqrt)


def _lerp(m: np.ndarray, g: np.ndarray, w: float) -> np.ndarray:
    wf = np.float32(w)
    d = (g - m).astype(np.float32)
    return _fma(wf, d, m) if abs(wf) < 0.5 else _fma(np.float32(wf - np.float32(1.0)), d, g)


def _sign(x: np.ndarray) -> np.ndarray:
    """torch.sign: (0 < x) - (x < 0), so 0 for NaN."""
    return ((x > 0).astype(np.float32) - (x < 0).astype(np.float32)).astype(np.float32)


def optrepo_init(opt: str, n: int, lr: float) -> Dict[str, object]:
    """The state torch creates at a parameter's first step (buffers and the
    per-parameter fp32 scalar tensors), before that step runs."""
    z = lambda: np.zeros(n, np.float32)  # noqa: E731
    st: Dict[str, object] = {name: z() for name in OPTREPO_STATE[opt]}
    if opt == "rprop":
        st["step_size"] = np.full(n, np.float32(lr), np.float32)
    if opt == "nadam":
        st["mu_product"] = np.float32(1.0)
    if opt == "asgd":
        st["eta"], st["mu"] = np.float32(lr), np.float32(1.0)
    return st


def fedopt_step(opt: str, p_old: np.ndarray, avg: np.ndarray, st: Dict[str, object], lr: float, step: int,
                sqrt: str = "torch") -> np.ndarray:
    """One server step of `opt` on one named parameter (1-based `step`); the
    state dict is updated in place, the new parameter returned."""
    p = np.ascontiguousarray(p_old, dtype=np.float32).reshape(-1).copy()
    a = np.ascontiguousarray(avg, dtype=np.float32).reshape(-1)
    g = (p - a).astype(np.float32)
    f = np.float32
    if opt in ("adamax", "nadam", "radam"):
        b1, b2, eps = 0.9, 0.999, 1e-8
        m = _lerp(st["exp_avg"], g, 1 - b1)
        st["exp_avg"] = m
        if opt == "adamax":  # adamax.py:277-303
            ei = np.maximum((st["exp_inf"] * f(b2)).astype(np.float32), (np.abs(g) + f(eps)).astype(np.float32))
            st["exp_inf"] = ei
            clr = lr / (1 - b1 ** step)
            return (p + (f(-clr) * m) / ei).astype(np.float32)
        v = _fma((f(1 - b2) * g).astype(np.float32), g, (st["exp_avg_sq"] * f(b2)).astype(np.float32))
        st["exp_avg_sq"] = v
        bc2 = 1 - b2 ** step
        if opt == "nadam":  # nadam.py:330-379, momentum_decay 4e-3
            mu = b1 * (1.0 - 0.5 * (0.96 ** (step * 4e-3)))
            mu_next = b1 * (1.0 - 0.5 * (0.96 ** ((step + 1) * 4e-3)))
            mp = f(st["mu_product"] * f(mu))
            st["mu_product"] = mp
            denom = (_sqrt((v / f(bc2)).astype(np.float32), sqrt) + f(eps)).astype(np.float32)
            p = (p + (f(-lr * (1.0 - mu) / (1.0 - float(mp))) * g) / denom).astype(np.float32)
            mpn = float(mp) * mu_next
            return (p + (f(-lr * mu_next / (1.0 - mpn)) * m) / denom).astype(np.float32)
        # radam.py:301-360
        bc1 = 1 - b1 ** step
        bcm = (m / f(bc1)).astype(np.float32)
        rho_inf = 2 / (1 - b2) - 1
        rho_t = rho_inf - 2 * step * (b2 ** step) / bc2
        x = (bcm * f(lr)).astype(np.float32)
        if rho_t > 5.0:
            rect = ((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t)) ** 0.5
            s = (_sqrt(v, sqrt) + f(eps)).astype(np.float32)
            adaptive = ((f(1.0) / s).astype(np.float32) * f(bc2 ** 0.5)).astype(np.float32)
            x = ((x * adaptive).astype(np.float32) * f(rect)).astype(np.float32)
        return (p - x).astype(np.float32)
    if opt == "adadelta":  # adadelta.py:281-302, rho 0.9, eps 1e-6
        rho, eps = 0.9, 1e-6
        sq = _fma((f(1 - rho) * g).astype(np.float32), g, (st["square_avg"] * f(rho)).astype(np.float32))
        std = _sqrt((sq + f(eps)).astype(np.float32), sqrt)
        delta = _sqrt((st["acc_delta"] + f(eps)).astype(np.float32), sqrt)
        delta = ((delta / std).astype(np.float32) * g).astype(np.float32)
        acc = _fma((f(1 - rho) * delta).astype(np.float32), delta, (st["acc_delta"] * f(rho)).astype(np.float32))
        st["square_avg"], st["acc_delta"] = sq, acc
        return _fma(delta, f(-lr), p)
    if opt == "asgd":  # asgd.py:247-275, lambd 1e-4, alpha 0.75, t0 1e6
        lambd, alpha, t0 = 1e-4, 0.75, 1e6
        eta = float(st["eta"])
        p = (p * f(1 - lambd * eta)).astype(np.float32)
        p = _fma(g, f(-eta), p)
        if float(st["mu"]) != 1:
            st["ax"] = (st["ax"] + ((p - st["ax"]).astype(np.float32) * st["mu"]).astype(np.float32)).astype(np.float32)
        else:
            st["ax"] = p.copy()
        st["eta"] = f(lr / ((1 + lambd * lr * step) ** alpha))
        st["mu"] = f(1 / max(1, step - t0))
        return p
    if opt == "rprop":  # rprop.py:257-291, etas (0.5, 1.2), step sizes (1e-6, 50)
        sgn = _sign((g * st["prev"]).astype(np.float32))
        sgn = np.where(sgn > 0, f(1.2), np.where(sgn < 0, f(0.5), f(1.0))).astype(np.float32)
        ss = np.clip((st["step_size"] * sgn).astype(np.float32), f(1e-6), f(50.0)).astype(np.float32)
        g2 = np.where(sgn == f(0.5), f(0.0), g).astype(np.float32)
        st["step_size"], st["prev"] = ss, g2
        return _fma((f(-1.0) * _sign(g2)).astype(np.float32), ss, p)
    raise ValueError(opt)


def fedopt_optrepo_round(opt: str, global_sd: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str],
                         raw_grad_list, lr: float, state: Dict[str, Dict[str, object]], step: int,
                         sqrt: str = "torch") -> "OrderedDict[str, torch.Tensor]":
    """One FedOptAPI round (fedopt_api.py:121-130) with server_optimizer =
    opt (adamax / nadam / radam / adadelta / asgd / rprop): FedAvg, the
    optimizer on named parameters (state[k] carries torch's per-parameter
    state across rounds, step is 1-based), averaged values for buffers."""
    class _A:
        federated_optimizer = "FedAvg"
    avg = agg(_A(), raw_grad_list)
    out = OrderedDict()
    for k, t_old in global_sd.items():
        if k in param_names:
            if k not in state:
                state[k] = optrepo_init(opt, t_old.numel(), lr)
            p = fedopt_step(opt, to_np(t_old).ravel(), to_np(avg[k]).ravel(), state[k], lr, step, sqrt=sqrt)
            out[k] = torch.from_numpy(p).reshape(t_old.shape)
        else:
            out[k] = avg[k].to(t_old.dtype).reshape(t_old.shape)
    return out


def fedopt_round(global_sd: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str],
                 raw_grad_list, lr: float, momentum: float,
                 mom_state: Dict[str, np.ndarray]) -> "OrderedDict[str, torch.Tensor]":
    """FedOptAggregator.aggregate (:81-116): FedAvg, then the SGD step on named
    parameters, averaged values for buffers (int64 buffers truncated by
    load_state_dict's copy_).  mom_state carries the momentum buffers across
    rounds (the optimizer state_dict round trip of :105-111)."""
    class _A:
        federated_optimizer = "FedAvg"
    avg = agg(_A(), raw_grad_list)
    out = OrderedDict()
    for k, t_old in global_sd.items():
        if k in param_names:
            first = k not in mom_state
            p, b = fedopt_sgd(to_np(t_old).ravel(), to_np(avg[k]).ravel(), mom_state.get(k), lr, momentum, first)
            if b is not None:
                mom_state[k] = b
            out[k] = torch.from_numpy(p).reshape(t_old.shape)
        else:
            out[k] = avg[k].to(t_old.dtype).reshape(t_old.shape)
    return out


# --------------------------------------------------------------------------
# Robust aggregation (core/security/defense)


def _is_weight_param(k: str) -> bool:
    """core/security/common/utils.py:16-21."""
    return "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k


def lower_median_cols(stack: np.ndarray) -> np.ndarray:
    """torch.median(x, dim=-1).values for x = stack.T ([M, K] -> [M]): element
    (K-1)//2 of each sorted column; a column with a NaN yields its first NaN
    (ATen's median: find_if(isnan) before nth_element).

    A zero median in a column holding both -0.0 and +0.0 takes its sign from
    the IEEE total order (-0 < +0), as the GPU kernels do.  torch's
    nth_element compares with `<`, so there the sign of that zero follows the
    column's input order (np.sort's choice is arbitrary as well): PARITY
    UNPINNED for that corner, the value (zero) is the same."""
    K = stack.shape[0]
    r = (K - 1) // 2
    srt = np.sort(stack, axis=0)  # NaNs sort last; they are overridden below
    med = srt[r].astype(stack.dtype)
    zc = np.nonzero(med == 0)[0]
    if zc.size:  # rank r falls among the column's zeros: -0 if it is within the negative zeros
        sub = stack[:, zc]
        below = (sub < 0).sum(axis=0) + ((sub == 0) & np.signbit(sub)).sum(axis=0)
        med[zc] = np.where(r < below, -0.0, 0.0).astype(stack.dtype)
    isn = np.isnan(stack)
    anyn = isn.any(axis=0)
    if anyn.any():
        first = np.argmax(isn, axis=0)
        med[anyn] = stack[first[anyn], np.nonzero(anyn)[0]]
    return med


def _exact_f32(t: torch.Tensor) -> np.ndarray:
    """Values as float32, exactly (bf16 bits widened, f16 / ints converted)."""
    a = to_np(t).ravel()
    if t.dtype == torch.bfloat16:
        return (a.astype(np.uint32) << 16).view(np.float32)
    return a.astype(np.float32)


def coordinate_wise_median(raw_grad_list):
    """CoordinateWiseMedianDefense.defend_on_aggregation
    (coordinate_wise_median_defense.py:18-44), including its walk over ALL of
    client 0's keys (misaligned for models with BN buffers -> RuntimeError)."""
    vecs = []
    for n, params in raw_grad_list:
        parts = [_exact_f32(v) for k, v in params.items() if _is_weight_param(k)]
        if not parts:
            raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")
        vecs.append(np.concatenate(parts))
    # torch.cat's promoted dtype (bf16 / f16 models stay 16-bit); the median
    # is one of the inputs, so selecting in fp32 and casting back is exact
    cat_dtype = torch.cat([v.reshape(-1)[:0] for k, v in raw_grad_list[0][1].items() if _is_weight_param(k)]).dtype
    med = torch.from_numpy(lower_median_cols(np.stack(vecs))).to(cat_dtype)
    index = 0
    (num0, averaged_params) = raw_grad_list[0]
    for k, params in list(averaged_params.items()):
        averaged_params[k] = med[index:index + params.numel()].view(params.size())
        index += params.numel()
    return averaged_params


def trimmed_mean(model_list, trimmed_num):
    """common/utils.py:213-228 (scores are the sample counts; stable sort)."""
    temp = sorted([(n, g, n) for n, g in model_list], key=lambda t: t[2])
    temp = temp[trimmed_num: len(model_list) - trimmed_num]
    return [(t[0], t[1]) for t in temp]


def weight_vector(params) -> np.ndarray:
    """vectorize_weight (core/security/common/utils.py:8-13) of an fp32 model."""
    return np.concatenate([to_np(v).astype(np.float32).ravel() for k, v in params.items() if _is_weight_param(k)])


def dist2(a: np.ndarray, b: np.ndarray) -> float:
    """Sum of the squares of the fp32 differences a - b (as the reference forms
    them), exactly squared and summed in fp64."""
    d = (a - b).astype(np.float32).astype(np.float64)
    return float(np.dot(d, d))


def fp32_norm(sq: float) -> float:
    """torch.norm(fp32 vector).item(): the root rounded to fp32."""
    return float(np.float32(np.sqrt(sq)))


def krum_select(raw_grad_list, byzantine_client_num: int, krum_param_m: int = 1):
    """KrumDefense.defend_before_aggregation (krum_defense.py:28-60): scores =
    sum of the K - f - 2 smallest `norm(v_i - v_j).item() ** 2`, fp32 argsort,
    the m best ORIGINAL tuples in score order.  Returns (list, scores)."""
    K = len(raw_grad_list)
    if not 2 * byzantine_client_num + 2 <= K - krum_param_m:
        raise ValueError("byzantine_client_num conflicts with requirements in Krum: "
                         "2 * byzantine_client_num + 2 < client number - krum_param_m")
    vecs = [weight_vector(p) for _, p in raw_grad_list]
    scores = []
    for i in range(K):
        ds = sorted(fp32_norm(dist2(vecs[i], vecs[j])) ** 2 for j in range(K) if j != i)
        scores.append(sum(ds[0:K - byzantine_client_num - 2]))
    order = torch.argsort(torch.Tensor(scores)).tolist()[0:krum_param_m]
    return [raw_grad_list[i] for i in order], scores


def norm_diff_clip(raw_grad_list, global_model, norm_bound: float):
    """NormDiffClippingDefense.defend_before_aggregation
    (norm_diff_clipping_defense.py:20-54): per client, d = fp32(local - global)
    over the weight keys, divisor c = max(1, norm(d) / bound) taken as fp32,
    weights = fp32(fp32(d / c) + global); other keys are the client's own."""
    g = weight_vector(global_model)
    out = []
    for n, local in raw_grad_list:
        v = weight_vector(local)
        d = (v - g).astype(np.float32)
        c = np.float32(max(1, fp32_norm(float(np.dot(d.astype(np.float64), d.astype(np.float64)))) / norm_bound))
        clipped = (d / c).astype(np.float32)
        new, idx = OrderedDict(), 0
        for k, t in local.items():
            if _is_weight_param(k):
                m = t.numel()
                gk = to_np(global_model[k]).astype(np.float32).ravel()
                new[k] = torch.from_numpy((clipped[idx:idx + m] + gk).astype(np.float32)).view(t.size())
                idx += m
            else:
                new[k] = t
        out.append((n, new))
    return out


def _f32(t: torch.Tensor) -> np.ndarray:
    """A tensor's values as float32 the way torch promotes int64 * float."""
    return to_np(t).astype(np.float32)


def mix_two(first, second, w_first: float, w_second: float):
    """`w_first * first[k] + w_second * second[k]` per key of `second`, in
    torch's fp32 arithmetic (each product rounded, then the sum)."""
    out = OrderedDict()
    for k, t in second.items():
        a = (np.float32(w_first) * _f32(first[k])).astype(np.float32)
        b = (np.float32(w_second) * _f32(t)).astype(np.float32)
        out[k] = torch.from_numpy(np.asarray(a + b, dtype=np.float32)).view(t.size())
    return out


def slsgd(args, raw_grad_list, global_model):
    """SLSGDDefense (slsgd_defense.py:28-67): bounds checks, option-2 trim by
    sample count, FedAvg, then (1 - alpha) * global + alpha * avg."""
    import math

    if args.alpha > 1 or args.alpha < 0:
        raise ValueError("the bound of alpha is [0, 1]")
    b = args.trim_param_b
    if b > math.ceil(len(raw_grad_list) / 2) - 1 or b < 0:
        raise ValueError("the bound of b")
    if args.option_type not in (1, 2):
        raise Exception("Such option type does not exist!")
    lst = trimmed_mean(raw_grad_list, b) if args.option_type == 2 else raw_grad_list
    return mix_two(global_model, agg(args, lst), 1 - args.alpha, args.alpha), lst


def bucketization(raw_grad_list, bucket_size: int):
    """common/bucket.py:6-28: per group of bucket_size consecutive clients the
    weighted average with w_i = n_i / sum n (the FedAvg chain, int keys ->
    float32), keys of client 0; the group's sample count."""
    import math

    K = len(raw_grad_list)
    keys = list(raw_grad_list[0][1].keys())
    out = []
    for b in range(math.ceil(K / bucket_size)):
        grp = raw_grad_list[b * bucket_size: min((b + 1) * bucket_size, K)]
        total = 0
        for n, _ in grp:
            total += n
        ws = [n / total for n, _ in grp]
        out.append((total, OrderedDict((k, wsum([p[k] for _, p in grp], ws)) for k in keys)))
    return out


def cclip(raw_grad_list, tau: float, bucket_size: int):
    """CClipDefense.defend_before_aggregation (cclip_defense.py:30-71); the
    caller seeds numpy's global RNG as the reference run did.  Returns (new
    list, initial guess dict)."""
    groups = bucketization(raw_grad_list, bucket_size)
    guess = groups[np.random.randint(0, len(groups))][1]
    g = weight_vector(guess)
    new = []
    for n, params in groups:
        score = min(1, tau / (fp32_norm(dist2(weight_vector(params), g)) + 1e-8))
        new.append((n, OrderedDict(
            (k, torch.from_numpy(np.asarray((_f32(t) - _f32(guess[k])).astype(np.float32) * np.float32(score),
                                            dtype=np.float32)).view(t.size())) for k, t in params.items())))
    return new, guess


def cclip_after(global_model, guess):
    """cclip_defense.py:57-60: guess[k] + global[k]."""
    return OrderedDict((k, torch.from_numpy(np.asarray(_f32(guess[k]) + _f32(t), dtype=np.float32)).view(t.size()))
                       for k, t in global_model.items())


def defended_agg(args, raw_grad_list, global_model=None):
    """FedMLDefender flow for the reduction and distance defenses
    (fedml_defender.py:131-171), followed by the base FedAvg operator."""
    if args.defense_type in ("krum", "multikrum"):
        m = getattr(args, "krum_param_m", None)
        sel, _ = krum_select(raw_grad_list, args.byzantine_client_num, m if isinstance(m, int) else 1)
        return agg(args, sel)
    if args.defense_type == "norm_diff_clipping":
        return agg(args, norm_diff_clip(raw_grad_list, global_model, args.norm_bound))
    if args.defense_type == "wise_median":
        return coordinate_wise_median(raw_grad_list)
    if args.defense_type == "trimmed_mean":
        if args.beta > 1 / 2 or args.beta < 0:
            raise ValueError("the bound of beta is [0, 1/2)")
        return agg(args, trimmed_mean(raw_grad_list, int(args.beta * len(raw_grad_list))))
    raise NotImplementedError(args.defense_type)


# --------------------------------------------------------------------------
# LightSecAgg field arithmetic


def finite_sum(weights_finite, p):
    """core/mpc/lightsecagg.py:134-148: w = x_0 ; w = (w + x_i) mod p (numpy
    int64: wrapping add, floor modulo)."""
    out = OrderedDict((k, np.array(v, dtype=np.int64, copy=True)) for k, v in weights_finite[0].items())
    for k in out:
        for d in weights_finite[1:]:
            with np.errstate(over="ignore"):
                out[k] = np.mod(out[k] + d[k], p)
    return out


def lsa_reconstruct(dicts, mask, p, q_bits):
    """lsa_fedml_aggregator.py:139-166 with lightsecagg.py:157-182 given the
    decoded aggregate mask (d, 1)."""
    out = OrderedDict()
    pos = 0
    K = len(dicts)
    for k in dicts[0]:
        s = np.array(dicts[0][k], dtype=np.int64, copy=True)
        for d in dicts[1:]:
            with np.errstate(over="ignore"):
                s = s + d[k]
        n = s.size
        with np.errstate(over="ignore"):
            s = s - np.asarray(mask).reshape(-1)[pos:pos + n].reshape(s.shape)
        pos += n
        xq = np.mod(s, p)
        v = np.where(xq.astype(np.float64) - (p - 1) / 2 > 0, xq.astype(np.float64) - float(p),
                     xq.astype(np.float64)) / float(2 ** q_bits)
        t = torch.from_numpy(np.asarray(v, dtype=np.float64).astype(np.float32).reshape(v.shape if v.ndim else (1,)))
        out[k] = t * (1 / K)
    return out


def robust_learning_rate(raw_grad_list, robust_threshold, base_aggregation_func=None):
    """RobustLearningRateDefense.run (core/security/defense/robust_learning_rate_defense.py:35-62):
    per key, the FedAvg chain (sample-count weights n_i / Σn) and the sum of the
    clients' torch.sign values; lr = |Σ sign|, set to -1 where below the
    threshold, then to 1 where at or above it (in that order), and the key
    becomes lr * avg.  Keys are rebound in client 0's dict, which is returned.
    robust_threshold == 0 hands the list to base_aggregation_func."""
    if robust_threshold == 0:
        return base_aggregation_func(raw_grad_list)
    total = 0
    for n, _ in raw_grad_list:
        total += n
    num0, avg_params = raw_grad_list[0]
    ws = [n / total for n, _ in raw_grad_list]
    thr = np.float32(robust_threshold)
    for k in list(avg_params.keys()):
        ts = [d[k] for _, d in raw_grad_list]
        avg = to_np(wsum(ts, ws)).astype(np.float32)
        sgn = np.zeros(avg.shape, dtype=np.float32)
        for t in ts:
            x = _f32(t)
            # torch.sign is (0 < x) - (x < 0): +0 for ±0 and for NaN (np.sign(NaN) is NaN)
            sgn = np.asarray(sgn + ((x > 0).astype(np.float32) - (x < 0).astype(np.float32)), dtype=np.float32)
        lr = np.abs(sgn)
        with np.errstate(invalid="ignore"):
            lr = np.where(lr < thr, np.float32(-1), lr)
            lr = np.where(lr >= thr, np.float32(1), lr)
        avg_params[k] = torch.from_numpy(np.asarray(lr * avg, dtype=np.float32)).view(ts[0].size())
    return avg_params
