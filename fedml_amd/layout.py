"""Row layout of one client's state dict: the shared contract of the HBM
bucket (fedml_amd.bucket) and the wire format (fedml_amd.wire).

Keys are grouped by storage dtype; inside a group every key starts at a
16-byte-aligned element offset, in the model's key order.  Integer keys are,
by default, stored in the float32 group as fl32(v) (torch computes
int64 * python_float as fl32(fl32(v) * fl32(w)), so the reduction is
bit-identical), which keeps a whole ResNet state dict in ONE row.
"""
from __future__ import annotations

import hashlib
import json
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

Entry = Tuple[str, Tuple[int, ...], torch.dtype]

INT_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
ROW_DTYPES = (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64)
ROW_ALIGN_ELEMS = 64  # rows padded to 64 elements (>= 128 B); keys 16-B aligned


def numel(shape) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n


def out_dtype(dt: torch.dtype) -> torch.dtype:
    """Result dtype of the weighted sum: int64 * python float -> float32."""
    return torch.float32 if dt == torch.int64 else dt


class Group:
    """Keys of one storage dtype packed into one row."""

    def __init__(self, dtype: torch.dtype):
        self.dtype = dtype
        self.out_dtype = out_dtype(dtype)
        self.esize = torch.empty((), dtype=dtype).element_size()
        self.keys: List[str] = []
        self.shapes: List[Tuple[int, ...]] = []
        self.offsets: List[int] = []
        self.numels: List[int] = []
        self.length = 0
        self.rows: Optional[torch.Tensor] = None     # set by ClientBucket
        self.d_ptrs: Optional[torch.Tensor] = None   # set by ClientBucket

    def add(self, key: str, shape) -> None:
        align = max(1, 16 // self.esize)
        start = (self.length + align - 1) // align * align
        n = numel(shape)
        self.keys.append(key)
        self.shapes.append(tuple(int(x) for x in shape))
        self.offsets.append(start)
        self.numels.append(n)
        self.length = start + n

    @property
    def padded(self) -> int:
        return (max(self.length, 1) + ROW_ALIGN_ELEMS - 1) // ROW_ALIGN_ELEMS * ROW_ALIGN_ELEMS


class RowLayout:
    def __init__(self, layout, promote_ints: bool = True):
        if isinstance(layout, dict):
            entries = [(k, tuple(t.shape), t.dtype) for k, t in layout.items()]
        else:
            entries = [(k, tuple(s), d) for k, s, d in layout]
        self.entries: List[Entry] = entries
        self.promote_ints = promote_ints
        self.groups: "OrderedDict[torch.dtype, Group]" = OrderedDict()
        self.where: Dict[str, Tuple[Group, int]] = {}
        self.int_keys = set()
        for key, shape, dt in entries:
            if dt in INT_DTYPES:
                self.int_keys.add(key)
                dt = torch.float32 if promote_ints else torch.int64
            if dt not in ROW_DTYPES:
                raise TypeError(f"key {key!r}: unsupported dtype {dt}")
            g = self.groups.get(dt)
            if g is None:
                g = self.groups[dt] = Group(dt)
            self.where[key] = (g, len(g.keys))
            g.add(key, shape)

    def signature(self) -> str:
        """sha256 of everything that fixes the byte layout."""
        desc = [[k, list(s), str(d)] for k, s, d in self.entries]
        return hashlib.sha256(json.dumps([1, self.promote_ints, desc]).encode()).hexdigest()

    def same_as(self, other: "RowLayout") -> bool:
        return self.signature() == other.signature()
