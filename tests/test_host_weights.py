"""Kernel-argument weights (fedml_amd.kernels.weights_for / HostWeights) on
the CPU: the exact fp32 / fp64 values the launch copies, and the reuse of the
last array built for the same values (a round over G shards or several dtype
groups builds it once; -0.0 and +0.0 are different weights)."""
from __future__ import annotations

import numpy as np
import torch

from fedml_amd import kernels as kn


def test_values_are_the_fp32_and_fp64_roundings():
    ws = [1 / 3, 2 / 3, 1e-40, -0.0]
    h32 = kn.weights_for(ws, torch.float32, None)
    h64 = kn.weights_for(ws, torch.float64, None)
    assert np.array(list(h32.buf), dtype=np.float32).tobytes() == np.array(ws, dtype=np.float32).tobytes()
    assert np.array(list(h64.buf), dtype=np.float64).tobytes() == np.array(ws, dtype=np.float64).tobytes()


def test_reuse_is_keyed_by_exact_values_and_dtype():
    a = kn.weights_for([0.25, 0.75], torch.float32, None)
    assert kn.weights_for([0.25, 0.75], torch.float32, None) is a
    assert kn.weights_for((0.25, np.float64(0.75)), torch.float32, None) is a  # same values, any sequence
    b = kn.weights_for([0.25, 0.75], torch.float64, None)
    assert b is not a and kn.weights_for([0.25, 0.75], torch.float32, None) is a  # one entry per dtype
    z = kn.weights_for([0.5, -0.0], torch.float32, None)
    p = kn.weights_for([0.5, 0.0], torch.float32, None)
    assert z is not p and np.signbit(z.buf[1]) and not np.signbit(p.buf[1])
    n1 = kn.weights_for([float("nan"), 1.0], torch.float32, None)
    assert kn.weights_for([float("nan"), 1.0], torch.float32, None) is n1  # same NaN bits: reused


def test_large_rounds_are_not_host_weights():
    import pytest

    with pytest.raises(ValueError):
        kn.HostWeights([0.0] * (kn.INLINE_MAX_K + 1))
