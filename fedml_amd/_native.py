"""ctypes binding of libfedagg.so (the C ABI in include/fedagg.h).

The library is built in-tree by ``python -m fedml_amd.build`` (or
``__graft_entry__.build()``) into ``fedml_amd/lib/libfedagg.so``.  There is no
fallback: if the library cannot be loaded every device entry point raises
``FedAggNativeError``.  torch is imported first so that libfedagg.so binds to
the HIP runtime torch already loaded (both carry SONAME libamdhip64.so.7), i.e.
one HIP runtime, one set of streams.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libfedagg.so")

FEDAGG_ALIGNED16 = 1
FEDAGG_HOST_WEIGHTS = 2
FEDAGG_ACC_REFERENCE = 0
FEDAGG_ACC_FP32 = 1

DT_F32, DT_BF16, DT_F16, DT_F64, DT_I64, DT_I32 = 0, 1, 2, 3, 4, 5
DIST_CHUNK, PAIR_CHUNK = 1024, 256  # FEDAGG_DIST_CHUNK / FEDAGG_PAIR_CHUNK
WORK_DIST2, WORK_PAIRDIST2, WORK_PAIRGRAM = 0, 1, 2
# FEDAGG_FEDOPT_*: the launch kinds of fedagg_wsum_fedopt_batch (besides the FEDAGG_OPT_* codes)
FEDOPT_AVG, FEDOPT_SGD, FEDOPT_ADAM, FEDOPT_ADAMW, FEDOPT_ADAGRAD, FEDOPT_RMSPROP = 0, 16, 17, 18, 19, 20


class FedOptLaunch(ctypes.Structure):
    """fedagg_fedopt_launch (include/fedagg.h), field for field."""
    _fields_ = [("d_src", ctypes.c_void_p), ("weights", ctypes.c_void_p), ("d_param", ctypes.c_void_p),
                ("d_state0", ctypes.c_void_p), ("d_state1", ctypes.c_void_p), ("scalars", ctypes.c_void_p),
                ("stream", ctypes.c_void_p), ("N", ctypes.c_int64), ("alpha", ctypes.c_double),
                ("lr", ctypes.c_float), ("momentum", ctypes.c_float), ("eps", ctypes.c_float),
                ("decay", ctypes.c_float), ("K", ctypes.c_int32), ("opt", ctypes.c_int32),
                ("device", ctypes.c_int32), ("first_step", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("dtype", ctypes.c_int32), ("acc_mode", ctypes.c_int32), ("reserved", ctypes.c_int32)]


# FEDAGG_OPT_*: the OptRepo optimizers of fedagg_wsum_fedopt_optrepo_f32
OPT_CODES = {"adamax": 1, "nadam": 2, "radam": 3, "adadelta": 4, "asgd": 5, "rprop": 6}

# Every symbol include/fedagg.h declares, with its ctypes signature.
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U32 = ctypes.c_uint32
_F = ctypes.c_float
SIGNATURES = {
    "fedagg_wsum_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_wsum_bf16": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _I32, _U32, _P]),
    "fedagg_wsum_bf16_f32out": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_wsum_f16": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _I32, _U32, _P]),
    "fedagg_round_f32": (ctypes.c_int, [_I32, _P, _I64, _P, _P]),
    "fedagg_wsum_f64": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_wsum_i64_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_sum": (ctypes.c_int, [_I32, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_wsum_muldiv": (ctypes.c_int, [_I32, _P, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_multi_blocks": (_I64, [_I32, _I64]),
    "fedagg_wsum_multi_f32": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _I32, _I64, _P]),
    "fedagg_wsum_multi": (ctypes.c_int, [_I32, _I32, _P, _P, _P, _P, _I32, _P, _I32, _I64, _P]),
    "fedagg_fedopt_sgd_f32": (ctypes.c_int, [_P, _P, _P, _I64, _F, _F, _I32, _P]),
    "fedagg_adam_scalars": (ctypes.c_int, [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          _I64, _P]),
    "fedagg_wsum_fedopt_adam_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _P, _I32, _U32, _P]),
    "fedagg_wsum_fedopt_sgd_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _F, _F, _I32, _U32, _P]),
    "fedagg_wsum_fedopt_adagrad_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _F, _F, _U32, _P]),
    "fedagg_wsum_fedopt_adamw_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _P, _F, _I32, _U32, _P]),
    "fedagg_wsum_fedopt_rmsprop_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _F, ctypes.c_double, _F, _U32,
                                                      _P]),
    "fedagg_optrepo_scalars": (ctypes.c_int, [_I32, ctypes.c_double, _I64, _P, _P]),
    "fedagg_wsum_fedopt_optrepo_f32": (ctypes.c_int, [_I32, _P, _P, _I32, _I64, _P, _P, _P, _P, _U32, _P]),
    "fedagg_wsum_fedopt_batch": (ctypes.c_int, [_P, _I32]),
    "fedagg_wsum_rlr_f32": (ctypes.c_int, [_P, _P, _I32, _I64, _F, _P, _U32, _P]),
    "fedagg_median_f32": (ctypes.c_int, [_P, _I32, _I64, _P, _U32, _P]),
    "fedagg_median": (ctypes.c_int, [_I32, _P, _I32, _I64, _P, _U32, _P]),
    "fedagg_sum_mod_i64": (ctypes.c_int, [_P, _I32, _I64, _I64, _P, _U32, _P]),
    "fedagg_lsa_reconstruct_f32": (ctypes.c_int, [_P, _I32, _I64, _P, _I64, _I32, _F, _P, _U32, _P]),
    "fedagg_host_pack": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32]),
    "fedagg_host_gather": (ctypes.c_int, [_P, _P, _P, _I32, _I32]),
    "fedagg_host_unpack": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32]),
    "fedagg_host_round_f32": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _P, _P]),
    "fedagg_device_round_f32": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _P, _P]),
    "fedagg_robust_work_len": (_I64, [_I32, _I32, _I64]),
    "fedagg_dist2_f32": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P, _I64, _P]),
    "fedagg_pairdist2_f32": (ctypes.c_int, [_P, _I32, _P, _I64, _P, _P, _I64, _P]),
    "fedagg_pairgram2_f32": (ctypes.c_int, [_P, _I32, _P, _I64, _P, _P, _I64, _P]),
    "fedagg_clip_diff_f32": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P]),
    "fedagg_scale_diff_f32": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P]),
    "fedagg_last_error": (ctypes.c_char_p, []),
    "fedagg_version": (_I32, []),
}


class FedAggNativeError(RuntimeError):
    """libfedagg.so is missing, failed to load, or a kernel call failed."""


_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return libfedagg.so; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise FedAggNativeError(
                    f"{LIB_PATH} not found: build it with `python -m fedml_amd.build` "
                    "(there is no CPU fallback)")
            try:
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
            except OSError as e:  # pragma: no cover - environment dependent
                raise FedAggNativeError(f"cannot load {LIB_PATH}: {e}") from e
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().fedagg_last_error().decode(errors="replace")
        raise FedAggNativeError(f"{what} failed (rc={rc}): {msg}")


def stream_handle(stream: "torch.cuda.Stream | None" = None) -> int:
    """Raw hipStream_t of a torch stream (default: the current stream)."""
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)
