"""include/fedagg.h promises stream-ordered, allocation-free entry points
that can be captured into a hipGraph: capture the round's launches once,
replay, and get the eager result bit for bit."""
from __future__ import annotations

import pytest
import torch

import golden_util as gu
from fedml_amd import defense as dfn
from fedml_amd.bucket import ClientBucket

pytestmark = pytest.mark.gpu


def test_reduction_and_median_replay_from_a_graph(cuda_device):
    K, N = 12, 100_003
    entries = [("w", (N,), torch.float32), ("b", (37,), torch.float32), ("c", (3,), torch.int64)]
    bucket = ClientBucket(entries, K, cuda_device)
    g = torch.Generator(device=cuda_device).manual_seed(11)
    for dt, grp in bucket.groups.items():
        grp.rows.normal_(0.0, 0.05, generator=g)
    ns = [100 + 37 * i for i in range(K)]
    w = bucket.weights(ns)
    grp = bucket.groups[torch.float32]
    eager = bucket.new_outputs()
    bucket.reduce_into(eager, w)  # weights ride in the kernel arguments (K <= 256): nothing to upload
    med_eager = torch.empty(grp.padded, device=cuda_device)
    dfn.median_rows(grp.d_ptrs, K, grp.length, med_eager, aligned=True)
    torch.cuda.synchronize()

    outs = bucket.new_outputs()
    med = torch.empty(grp.padded, device=cuda_device)
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda_device)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            bucket.reduce_into(outs, w)
            dfn.median_rows(grp.d_ptrs, K, grp.length, med, aligned=True)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    gu.assert_same(outs[torch.float32][:grp.length].cpu(), eager[torch.float32][:grp.length].cpu(), "wsum")
    gu.assert_same(med[:grp.length].cpu(), med_eager[:grp.length].cpu(), "median")
