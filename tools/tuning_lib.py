"""The tuning build of libfedagg (tools only; never shipped or imported by fedml_amd).

The A/B entry points the shipped tile shapes were chosen from
(fedagg_wsum_f32_variant, fedagg_wsum_tiny_variant and their name / count
queries) are compiled only with -DFEDAGG_TUNING.  This module builds
csrc/fedagg.hip that way into tools/_build/libfedagg_tuning.so, linked with the
product's own median / robust objects, and loads it with the product ABI's
ctypes signatures plus the tuning ones:

    python -m tools.tuning_lib          # build
    from tools.tuning_lib import lib, check

The tuning entries (csrc/fedagg.hip, FEDAGG_TUNING):
    int fedagg_wsum_f32_variant(const float* const* d_src, const float* d_w, int32_t K, int64_t N,
                                float* d_out, int32_t variant, fedagg_stream_t stream);
    const char* fedagg_variant_name(int32_t variant);
    int32_t fedagg_num_variants(void);
    int fedagg_wsum_tiny_variant(int32_t dtype, const void* const* d_src, const float* d_w, int32_t K,
                                 int64_t N, void* d_out, int32_t variant, fedagg_stream_t stream);
        dtype: FEDAGG_DT_F32, FEDAGG_DT_BF16 (reference chain), TUNE_BF16_F32OUT (bf16 rows, fp32
        partial out) or TUNE_BF16_ACC32 (bf16 rows, fp32 accumulation); pointers 16-byte aligned,
        d_w a device array
    const char* fedagg_tiny_variant_name(int32_t variant);
    int32_t fedagg_num_tiny_variants(void);
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fedml_amd import _native as nat  # noqa: E402
from fedml_amd import build as fbuild  # noqa: E402

OUT_DIR = os.path.join(ROOT, "tools", "_build")
OUT = os.path.join(OUT_DIR, "libfedagg_tuning.so")
TUNE_BF16_F32OUT, TUNE_BF16_ACC32 = 0x101, 0x102

_P, _I32, _I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
TUNING_SIGNATURES = {
    "fedagg_wsum_f32_variant": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _I32, _P]),
    "fedagg_variant_name": (ctypes.c_char_p, [_I32]),
    "fedagg_num_variants": (_I32, []),
    "fedagg_wsum_tiny_variant": (ctypes.c_int, [_I32, _P, _P, _I32, _I64, _P, _I32, _P]),
    "fedagg_tiny_variant_name": (ctypes.c_char_p, [_I32]),
    "fedagg_num_tiny_variants": (_I32, []),
}


def build(force: bool = False) -> str:
    fbuild.build()  # the product objects (median, robust) this links with
    src = fbuild.SRC
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(
            os.path.getmtime(p) for p in (src, fbuild.HEADER, fbuild.OUT, __file__)):
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    obj = os.path.join(OUT_DIR, "fedagg_tuning.o")
    subprocess.run([fbuild.hipcc(), *fbuild.HIPCC_FLAGS, "-DFEDAGG_TUNING", "-c", "-o", obj, src], check=True)
    others = [fbuild._obj(s) for s in fbuild.SRCS if s != src]
    subprocess.run([fbuild.hipcc(), f"--offload-arch={fbuild.ARCH}", "-shared", "-fPIC", "-o", OUT, obj, *others],
                   check=True)
    return OUT


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        handle = ctypes.CDLL(build(), mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in {**nat.SIGNATURES, **TUNING_SIGNATURES}.items():
            fn = getattr(handle, name)
            fn.restype, fn.argtypes = res, args
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise nat.FedAggNativeError(f"{what} failed (rc={rc}): {lib().fedagg_last_error().decode(errors='replace')}")


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
