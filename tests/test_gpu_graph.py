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


@pytest.mark.parametrize("K,N,acc", [(256, (8 << 20) - 12_345, "reference"), (40, 8 << 20, "fp32"),
                                     (40, 1 << 20, "reference")])
def test_bf16_tiles_replay_from_a_graph(K, N, acc, cuda_device):
    """The bf16 dispatch reads the device's CU count (tile shape by the fill
    of the last resident round): captured launches replay bit for bit."""
    from fedml_amd import kernels as kn

    L = (N + 63) // 64 * 64  # 16-byte aligned rows: the launches below say FEDAGG_ALIGNED16
    rows = torch.empty((K, L), dtype=torch.bfloat16, device=cuda_device).normal_(0.0, 0.05)
    ptrs = torch.tensor([rows[i].data_ptr() for i in range(K)], dtype=torch.int64, device=cuda_device)
    w = kn.weights_for([1.0 / K + 1e-4 * i for i in range(K)], torch.bfloat16, cuda_device)
    mode = {"reference": kn.ACC_REFERENCE, "fp32": kn.ACC_FP32}[acc]
    eager = torch.empty(N, dtype=torch.bfloat16, device=cuda_device)
    kn.wsum_ptrs(torch.bfloat16, ptrs, w, K, N, eager, True, mode)
    torch.cuda.synchronize()
    out = torch.empty_like(eager)
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda_device)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            kn.wsum_ptrs(torch.bfloat16, ptrs, w, K, N, out, True, mode)
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), eager.view(torch.int16))
