"""LightSecAgg field arithmetic: oracle pinned to the reference (CPU) and the
HIP kernels against the same golden vectors (GPU)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from oracle import fedavg_oracle as orc

NAMES = [c["name"] for c in cases.SECAGG_CASES]


def _oracle(spec):
    dicts, mask = cases.secagg_inputs(spec)
    if spec["kind"] == "finite_sum":
        return OrderedDict((k, torch.from_numpy(np.asarray(v))) for k, v in orc.finite_sum(dicts, spec["p"]).items())
    return orc.lsa_reconstruct(dicts, mask, spec["p"], spec["q"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference(name):
    meta, arrays = gu.load(name)
    gu.assert_groups(_oracle(meta["spec"]), meta, arrays, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_reference(name, cuda_device):
    from fedml_amd import secagg

    meta, arrays = gu.load(name)
    spec = meta["spec"]
    dicts, mask = cases.secagg_inputs(spec)
    if spec["kind"] == "finite_sum":
        res = secagg.aggregate_models_in_finite(dicts, spec["p"])
        res = OrderedDict((k, torch.from_numpy(np.asarray(v))) for k, v in res.items())
    else:
        md = {i: d for i, d in enumerate(dicts)}
        res = secagg.model_reconstruction(md, list(range(spec["K"])), mask, spec["p"], spec["q"])
        assert res is md[0]
    gu.assert_groups(res, meta, arrays, name)
