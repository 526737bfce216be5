"""Synthetic client updates of a given state-dict structure.

Recipe: per key, base ~ N(0, 0.05²) and client_i = base + 0.01·ε_i; sample
counts n_i ~ U{100..1000}; int64 entries (BatchNorm num_batches_tracked) are
round_idx + i.  Host inputs come from numpy's PCG64 stream (stable across
machines, so the golden fixtures can store seeds instead of megabytes of
inputs); device inputs for the benchmark are generated directly in HBM.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Sequence, Tuple

import numpy as np
import torch

from .shapes import Entry


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[np.isnan(x)] = 0x7FC0
    return r


def _to_tensor(x: np.ndarray, dtype: torch.dtype, shape) -> torch.Tensor:
    if dtype == torch.bfloat16:
        return torch.from_numpy(_bf16_bits(x).view(np.int16)).view(torch.bfloat16).reshape(shape)
    if dtype == torch.float16:
        return torch.from_numpy(x.astype(np.float16)).reshape(shape)
    if dtype == torch.float64:
        return torch.from_numpy(x.astype(np.float64)).reshape(shape)
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).reshape(shape)


def host_clients(entries: Sequence[Entry], K: int, seed: int, round_idx: int = 0,
                 sample_nums: Sequence[float] | None = None,
                 int_range: Tuple[int, int] | None = None) -> List[Tuple[int, "OrderedDict[str, torch.Tensor]"]]:
    """K clients as the reference receives them: [(n_i, OrderedDict of CPU tensors)]."""
    rng = np.random.default_rng(seed)
    ns = list(sample_nums) if sample_nums is not None else [int(v) for v in rng.integers(100, 1001, K)]
    dicts: List["OrderedDict[str, torch.Tensor]"] = [OrderedDict() for _ in range(K)]
    for key, shape, dtype in entries:
        size = int(np.prod(shape)) if len(shape) else 1
        if dtype in (torch.int64, torch.int32):
            for i in range(K):
                if int_range is None:
                    v = np.full(size, round_idx + i, dtype=np.int64)
                else:
                    v = rng.integers(int_range[0], int_range[1], size, dtype=np.int64)
                dicts[i][key] = torch.from_numpy(v.astype(np.int64)).reshape(shape).to(dtype)
            continue
        base = rng.standard_normal(size, dtype=np.float32) * np.float32(0.05)
        for i in range(K):
            x = base + np.float32(0.01) * rng.standard_normal(size, dtype=np.float32)
            dicts[i][key] = _to_tensor(x, dtype, shape)
    return [(ns[i], dicts[i]) for i in range(K)]


def fingerprint(raw: Sequence[Tuple[float, "OrderedDict[str, torch.Tensor]"]]) -> str:
    """sha256 over every input byte and sample count (fixture drift check)."""
    import hashlib

    h = hashlib.sha256()
    for item in raw:
        h.update(repr(item[0]).encode())
        for d in item[1:]:
            for k, t in d.items():
                h.update(k.encode())
                tt = t.detach().cpu().contiguous()
                if tt.dtype == torch.bfloat16:
                    tt = tt.view(torch.int16)
                h.update(tt.numpy().tobytes())
    return h.hexdigest()


def device_bucket(K: int, N: int, device, dtype: torch.dtype = torch.float32, seed: int = 0,
                  row_align: int = 64) -> torch.Tensor:
    """A [K, N_row] device tensor (rows padded to row_align elements) filled with
    the same recipe, generated in HBM (used by bench.py: 13 GB at config 3)."""
    gen = torch.Generator(device=device).manual_seed(seed)
    row = (N + row_align - 1) // row_align * row_align
    out = torch.empty((K, row), dtype=dtype, device=device)
    base = torch.randn(N, generator=gen, device=device, dtype=torch.float32) * 0.05
    tmp = torch.empty(N, device=device, dtype=torch.float32)
    for i in range(K):
        tmp.normal_(0.0, 1.0, generator=gen)
        out[i, :N].copy_(base + 0.01 * tmp)
        if row > N:
            out[i, N:].zero_()
    return out


def sample_nums(K: int, seed: int = 1) -> List[int]:
    rng = np.random.default_rng(seed)
    return [int(v) for v in rng.integers(100, 1001, K)]
