"""Loading golden fixtures and comparing results bit for bit."""
from __future__ import annotations

import glob
import json
import os
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np
import torch

FIX_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")

_NP = {"float32": np.float32, "float64": np.float64, "float16": np.float16, "int64": np.int64,
       "int32": np.int32, "bfloat16": np.uint16}
_TORCH = {"float32": torch.float32, "float64": torch.float64, "float16": torch.float16, "int64": torch.int64,
          "int32": torch.int32, "bfloat16": torch.bfloat16}


def fixture_names(prefix: str = "") -> List[str]:
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(FIX_DIR, f"{prefix}*.npz")))


def load(name: str) -> Tuple[dict, Dict[str, np.ndarray]]:
    with np.load(os.path.join(FIX_DIR, f"{name}.npz"), allow_pickle=False) as z:
        meta = json.loads(str(z["meta"]))
        arrays = {n: z[f"a{i}"] for i, n in enumerate(meta["array_names"])}
    return meta, arrays


def to_tensor(a: np.ndarray, dtype: str, shape) -> torch.Tensor:
    if dtype == "bfloat16":
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).reshape(shape)
    return torch.from_numpy(a.copy()).reshape(shape)


def expected_groups(meta, arrays) -> List["OrderedDict[str, torch.Tensor]"]:
    groups: List[OrderedDict] = []
    for o in meta["outputs"]:
        while len(groups) <= o["group"]:
            groups.append(OrderedDict())
        groups[o["group"]][o["key"]] = to_tensor(arrays[f"o{o['group']}:{o['key']}"], o["dtype"], o["shape"])
    return groups


def bits(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    if t.dtype == torch.float16:
        return t.view(torch.int16).numpy().view(np.uint16)
    if t.dtype == torch.float32:
        return t.numpy().view(np.uint32)
    if t.dtype == torch.float64:
        return t.numpy().view(np.uint64)
    return t.numpy()


def assert_same(actual: torch.Tensor, expected: torch.Tensor, what: str = "", zero_sign: bool = True) -> int:
    """Bit-identical, except that any NaN matches any NaN (payloads are not part
    of torch's contract either).  zero_sign=False also lets -0.0 match +0.0:
    the known divergence of a zero median whose column holds both zero signs
    (torch's nth_element returns whichever its input order puts at the rank;
    DESIGN.md §5b).  Returns the number of elements that differed only in the
    sign of a zero."""
    assert actual.dtype == expected.dtype, f"{what}: dtype {actual.dtype} != {expected.dtype}"
    assert tuple(actual.shape) == tuple(expected.shape), f"{what}: shape {actual.shape} != {expected.shape}"
    signs = 0
    if not zero_sign and actual.is_floating_point():
        av, ev = actual.detach().cpu().float(), expected.float()
        both_zero = (av == 0) & (ev == 0)
        signs = int((both_zero & (torch.signbit(av) != torch.signbit(ev))).sum())
        actual = torch.where(both_zero.to(actual.device), torch.zeros_like(actual), actual)
        expected = torch.where(both_zero, torch.zeros_like(expected), expected)
    a, e = bits(actual).ravel(), bits(expected).ravel()
    pos = np.arange(a.size)
    if actual.is_floating_point():
        an = torch.isnan(actual.detach().cpu().float()).numpy().ravel()
        en = torch.isnan(expected.float()).numpy().ravel()
        assert np.array_equal(an, en), f"{what}: NaN positions differ"
        a, e, pos = a[~an], e[~en], pos[~an]
    bad = np.nonzero(a != e)[0]
    if bad.size:
        j = int(pos[bad[0]])  # the element's index in the tensor (NaNs were left out of a / e)
        raise AssertionError(f"{what}: {bad.size} of {a.size} elements differ; first at {j}: "
                             f"got {actual.detach().cpu().reshape(-1)[j].item()!r} "
                             f"want {expected.reshape(-1)[j].item()!r}")
    return signs


def assert_groups(actual, meta, arrays, what="", zero_sign: bool = True) -> int:
    """Every output group against the fixture (assert_same); returns the
    count of zero-sign-only differences (zero_sign=False)."""
    exp = expected_groups(meta, arrays)
    got = list(actual) if isinstance(actual, tuple) else [actual]
    assert bool(meta.get("tuple")) == isinstance(actual, tuple), f"{what}: tuple-ness differs"
    assert len(got) == len(exp)
    signs = 0
    for g, (gd, ed) in enumerate(zip(got, exp)):
        assert list(gd.keys()) == list(ed.keys()), f"{what}: key order differs"
        for k in ed:
            signs += assert_same(gd[k], ed[k], f"{what}[{g}][{k}]", zero_sign)
    return signs


def snapshot_third(raw):
    """(tensor objects, clones) of client 0's second dict of a 3-tuple round."""
    if len(raw[0]) < 3:
        return None
    objs = dict(raw[0][2])
    return objs, {k: t.clone() for k, t in objs.items()}


def assert_third_mutation(snap, meta, arrays, what="") -> None:
    """SCAFFOLD's in-place `total_c_delta_para[k] += c_delta_para[k]`
    (agg_operator.py:110,113): which of client 0's c_delta tensors the
    reference mutated, and their values afterwards."""
    if snap is None or "client0_third_tensors_mutated" not in meta:
        return
    objs, before = snap
    want = set(meta["client0_third_tensors_mutated"])
    names = meta["array_names"]
    for k, t in objs.items():
        t = t.cpu()
        if t.is_floating_point() and torch.isnan(t).any():
            continue
        changed = not torch.equal(t, before[k].cpu())
        assert changed == (k in want), f"{what}: c_delta[{k}] mutated={changed}"
        if k in want:
            a = arrays[f"m2:{k}"]
            e = to_tensor(a, str(t.dtype).replace("torch.", ""), t.shape)
            assert_same(t, e, f"{what}: c_delta[{k}] after the call")
