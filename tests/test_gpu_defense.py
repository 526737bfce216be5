"""GPU parity of the robust-aggregation defenses against the reference's own
CoordinateWiseMedianDefense / CoordinateWiseTrimmedMeanDefense (golden)."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pytest
import torch

import cases
import golden_util as gu
from fedml_amd import defense as dfn
from fedml_amd import kernels as kn
from fedml_amd.server_aggregator import MI355XServerAggregator
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu


def _run(spec, raw):
    args = cases.DefenseArgs(spec)
    agg = MI355XServerAggregator(torch.nn.Linear(1, 1), args)
    lst, idxs = agg.on_before_aggregation(raw)
    assert idxs == list(range(len(raw)))
    return agg.on_after_aggregation(agg.aggregate(lst))


@pytest.mark.parametrize("device_inputs", [False, True])
@pytest.mark.parametrize("name", [c["name"] for c in cases.DEFENSE_CASES])
def test_defense_matches_reference(name, device_inputs, cuda_device):
    meta, arrays = gu.load(name)
    spec = meta["spec"]
    raw = cases.build_inputs(spec)
    if device_inputs:
        raw = [(n, OrderedDict((k, t.to(cuda_device)) for k, t in d.items())) for n, d in raw]
    if meta["error"]:
        with pytest.raises(Exception) as ei:
            _run(spec, raw)
        assert type(ei.value).__name__ == meta["error"]
        return
    res = _run(spec, raw)
    for t in res.values():
        assert t.is_cuda == device_inputs
    got = OrderedDict((k, t.cpu()) for k, t in res.items())
    if spec.get("signed_zero_ties"):
        # the known divergence: zero medians equal, their sign
        # the IEEE total order's; the kernels agree with the oracle bit for bit
        gu.assert_groups(got, meta, arrays, name, zero_sign=False)
        exp = orc.defended_agg(cases.DefenseArgs(spec), cases.build_inputs(spec))
        for k in exp:
            gu.assert_same(got[k], exp[k], f"{name}[{k}] vs oracle")
        return
    gu.assert_groups(got, meta, arrays, name)


@pytest.mark.parametrize("K", [1, 2, 7, 8, 9, 16, 17, 24, 33, 48, 64, 65, 96, 97, 100, 127, 128])
def test_median_kernel_vs_oracle(K, cuda_device):
    """Every KMAX bucket (full and padded kernels), with duplicates and
    infinities."""
    N = 20_011
    g = torch.Generator(device=cuda_device).manual_seed(K)
    rows = torch.randint(-50, 50, (K, N), generator=g, device=cuda_device).float() * 0.125
    rows[:, :7] = float("inf")
    rows[:, 7:9] = -float("inf")
    rows[K // 2, 100:110] = float("nan")
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, device=cuda_device)
    dfn.median_f32(d_ptrs, K, N, out)
    exp = orc.lower_median_cols(rows.cpu().numpy())
    gu.assert_same(out.cpu(), torch.from_numpy(exp), f"median K={K}")


def test_median_headline_shape_sampled(cuda_device):
    """128 clients x 25.6M fp32: 200,000 random columns vs the oracle."""
    K, N = 128, 25_610_152
    g = torch.Generator(device=cuda_device).manual_seed(3)
    rows = torch.empty((K, (N + 63) // 64 * 64), device=cuda_device)
    for i in range(K):
        rows[i].normal_(0.0, 0.05, generator=g)
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, device=cuda_device)
    dfn.median_f32(d_ptrs, K, N, out)
    idx = torch.randint(0, N, (200_000,), generator=torch.Generator().manual_seed(2)).to(cuda_device)
    exp = orc.lower_median_cols(rows[:, idx].cpu().numpy())
    gu.assert_same(out[idx].cpu(), torch.from_numpy(exp), "median headline")


@pytest.mark.parametrize("K", [129, 200, 255, 256, 257, 512, 700, 1024])
def test_median_lanes_kernel_vs_oracle(K, cuda_device):
    """More than 128 clients (4 or 8 lanes per column, register sorts plus
    cross-lane merges): full and padded kernels of every lane count, a ragged
    last workgroup, with duplicates, infinities, NaN columns and -0.0."""
    N = 3_001
    g = torch.Generator(device=cuda_device).manual_seed(K)
    rows = torch.randint(-50, 50, (K, N), generator=g, device=cuda_device).float() * 0.125
    rows[:, 17:29] = torch.randn(K, 12, generator=g, device=cuda_device)  # distinct values
    rows[:, :7] = float("inf")
    rows[:, 7:9] = -float("inf")
    rows[K // 2, 100:110] = float("nan")
    rows[K - 1, 105:115] = -float("nan")
    rows[:, 200:203] = -0.0
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, device=cuda_device)
    dfn.median_f32(d_ptrs, K, N, out)
    exp = orc.lower_median_cols(rows.cpu().numpy())
    gu.assert_same(out.cpu(), torch.from_numpy(exp), f"median K={K}")


def test_median_lanes_large_sampled(cuda_device):
    """512 clients x 4M fp32 (the config-4 client count): 100,000 random
    columns plus the ragged tail against the oracle."""
    K, N = 512, 4_000_037
    g = torch.Generator(device=cuda_device).manual_seed(5)
    rows = torch.randn((K, N), generator=g, device=cuda_device) * 0.05
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, device=cuda_device)
    dfn.median_f32(d_ptrs, K, N, out)
    idx = torch.cat([torch.randint(0, N, (100_000,), generator=torch.Generator().manual_seed(4)),
                     torch.arange(N - 40, N)]).to(cuda_device)
    exp = orc.lower_median_cols(rows[:, idx].cpu().numpy())
    gu.assert_same(out[idx].cpu(), torch.from_numpy(exp), "median K=512 sampled")


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [1025, 1500, 2048, 2049, 2561, 3000, 4096, 4097])
def test_median_more_than_1024_clients(aligned, dtype, K, cuda_device):
    """No client bound, as torch.median has none (coordinate_wise_median_
    defense.py:24-32): up to 4096 clients the 16- and 32-lane group kernels
    (packed for aligned 16-bit rows; widening rows take the radix select
    between 2049 and 2560), above that the radix-select kernel; every dtype,
    with duplicates, infinities, NaN columns (first NaN in client order) and
    -0.0, a ragged last tile and an odd column count."""
    N = 1_037
    g = torch.Generator(device=cuda_device).manual_seed(K)
    vals = (torch.randint(-50, 50, (K, N), generator=g, device=cuda_device).float() * 0.125).to(dtype)
    if aligned:  # 256-B row stride, as bucket rows have
        rows = torch.empty((K, 1_088), dtype=dtype, device=cuda_device)[:, :N]
        rows.copy_(vals)
    else:
        rows = vals
    rows[:, 17:29] = torch.randn(K, 12, generator=g, device=cuda_device).to(dtype)
    rows[:, :7] = float("inf")
    rows[:, 7:9] = -float("inf")
    rows[K // 2, 100:110] = float("nan")
    rows[K - 1, 105:115] = -float("nan")
    rows[:, 200:203] = -0.0
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    dfn.median_rows(d_ptrs, K, N, out, aligned=aligned)
    exp = torch.from_numpy(orc.lower_median_cols(rows.float().cpu().numpy())).to(dtype)
    gu.assert_same(out.cpu(), exp, f"median {dtype} K={K}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_median_more_than_2_30_columns(dtype, cuda_device):
    """A row longer than 2^30 elements (a whole-model stack past a billion
    parameters): the 32-bit-offset kernels run in chunks of 2^30 columns;
    columns on both sides of the chunk boundary and the ragged end vs the
    oracle."""
    K, N = 3, (1 << 30) + 4_099
    g = torch.Generator(device=cuda_device).manual_seed(30)
    L = (N + 127) // 64 * 64  # 256-B row stride: aligned rows, as bucket rows are
    rows = torch.empty((K, L), dtype=dtype, device=cuda_device)
    for i in range(K):
        rows[i].copy_(torch.randint(-1000, 1000, (L,), generator=g, device=cuda_device, dtype=torch.int32)
                      .to(dtype) * 0.001)
    rows = rows[:, :N]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    idx = torch.cat([torch.arange(0, 64), torch.arange((1 << 30) - 64, (1 << 30) + 64), torch.arange(N - 64, N),
                     torch.randint(0, N, (20_000,), generator=torch.Generator().manual_seed(1))]).to(cuda_device)
    exp = torch.from_numpy(orc.lower_median_cols(rows[:, idx].float().cpu().numpy())).to(dtype)
    gu.assert_same(out[idx].cpu(), exp, f"median {dtype} N > 2^30")
    del rows, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [1, 9, 33, 64, 127, 128, 129, 200, 256, 257, 384, 511, 512, 513, 700, 1000, 1024])
def test_median_16bit_rows_vs_oracle(aligned, dtype, K, cuda_device):
    """bf16 / f16 rows (a 16-bit model's stack): every kernel family (aligned
    rows with K <= 128 take the packed two-columns-per-lane kernel, with an odd
    last column), with duplicates, infinities, NaN columns (a NaN in only one
    column of a packed pair too) and -0.0; the result is the selected input,
    bit for bit."""
    N = 2_051
    g = torch.Generator(device=cuda_device).manual_seed(K + 7)
    vals = (torch.randint(-50, 50, (K, N), generator=g, device=cuda_device).float() * 0.125).to(dtype)
    if aligned:  # 256-B row stride, as bucket rows have
        rows = torch.empty((K, 2_112), dtype=dtype, device=cuda_device)[:, :N]
        rows.copy_(vals)
    else:
        rows = vals
    rows[:, 17:29] = torch.randn(K, 12, generator=g, device=cuda_device).to(dtype)
    rows[:, :7] = float("inf")
    rows[:, 7:9] = -float("inf")
    rows[K // 2, 100:110] = float("nan")
    rows[:, 200:203] = -0.0
    rows[K - 1, 301] = float("nan")  # odd column of a pair: its neighbour stays a plain median
    rows[0, N - 1] = float("nan")    # the unpaired last column
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    dfn.median_rows(d_ptrs, K, N, out, aligned=aligned)
    exp = torch.from_numpy(orc.lower_median_cols(rows.float().cpu().numpy())).to(dtype)
    gu.assert_same(out.cpu(), exp, f"median {dtype} K={K}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [129, 256, 300, 512, 513, 1000])
def test_median_16bit_streamed_many_column_blocks(dtype, K, cuda_device):
    """The streamed bit-plane kernels (aligned 16-bit rows, 128 < K <= 1024)
    over far more column blocks than resident blocks, so every block walks a
    range of them with its next tile's DMA in flight: sampled columns at the
    range seams, NaN columns (first NaN in client order, payload included) in
    many column blocks, infinities, -0.0 and the ragged end vs the oracle."""
    N = 400_003
    g = torch.Generator(device=cuda_device).manual_seed(K + 11)
    rows = torch.empty((K, (N + 127) // 128 * 128), dtype=dtype, device=cuda_device)[:, :N]
    rows.copy_((torch.randint(-300, 300, (K, N), generator=g, device=cuda_device).float() * 0.01).to(dtype))
    r16 = rows.view(torch.int16)
    nan = 0x7f80 if dtype == torch.bfloat16 else 0x7c00
    nan_cols = torch.arange(5, N, 9_973, device=cuda_device)
    late, early = K - 2, K // 2 + 1
    r16[late, nan_cols] = nan | 0x11
    r16[early, nan_cols[::2]] = ((nan | 0x23) | 0x8000) - 0x10000
    inf_cols = torch.arange(17, N, 7_919, device=cuda_device)
    rows[: K // 2 + 1, inf_cols] = float("inf")
    rows[:, inf_cols + 1] = -0.0
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    seams = torch.arange(0, N, 64 * ((N // 64 + 511) // 512), device=cuda_device)
    idx = torch.cat([seams, seams + 1, seams + 63, nan_cols, inf_cols, inf_cols + 1,
                     torch.arange(N - 300, N, device=cuda_device),
                     torch.randint(0, N, (8_000,), generator=g, device=cuda_device)]).clamp(max=N - 1).unique()
    exp = torch.from_numpy(orc.lower_median_cols(rows[:, idx].float().cpu().numpy())).to(dtype)
    gu.assert_same(out[idx].cpu(), exp, f"median {dtype} K={K} streamed")
    o16 = out.view(torch.int16)[nan_cols].cpu()
    want = torch.tensor([((nan | 0x23) | 0x8000) - 0x10000 if i % 2 == 0 else nan | 0x11
                         for i in range(len(nan_cols))], dtype=torch.int16)
    assert torch.equal(o16, want)
    del rows, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K,N", [(100, 1_001), (128, 998), (256, 1_000), (512, 999), (700, 65), (1024, 1),
                                 (2048, 77), (4096, 33)])
def test_median_16bit_lanes_first_nan_payload(dtype, K, N, cuda_device):
    """The packed lane-group kernel (16-bit rows, 128 < K <= 4096): a NaN
    column returns ITS FIRST NaN in client order, payload included, per half of
    a packed pair, when the NaNs sit in different lanes of the column group;
    an odd N takes the lone-last-column launch (N = 1: that launch alone)."""
    g = torch.Generator(device=cuda_device).manual_seed(K)
    rows = torch.empty((K, (N + 127) // 128 * 128), dtype=dtype, device=cuda_device)[:, :N]
    rows.copy_(torch.randn(K, N, generator=g, device=cuda_device).to(dtype))
    r16 = rows.view(torch.int16)
    nan = 0x7f80 if dtype == torch.bfloat16 else 0x7c00
    late, early = K - 3, K // 3 + 1  # different lanes of the group; the earlier client wins
    cols = [c for c in (0, 1, 2, 5, N - 1) if c < N]
    for c in cols:
        r16[late, c] = nan | 0x11
        r16[early, c] = ((nan | 0x23) | 0x8000) - 0x10000  # negative NaN, payload 0x23
    if N > 5:
        r16[late, 3] = nan | 0x5  # only one NaN: its pair neighbour (column 2) has two
    out = torch.empty(N, dtype=dtype, device=cuda_device)
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    o16 = out.view(torch.int16).cpu()
    for c in cols:
        assert int(o16[c]) & 0xffff == (nan | 0x23) | 0x8000, f"column {c}: {int(o16[c]) & 0xffff:#06x}"
    if N > 5:
        assert int(o16[3]) & 0xffff == nan | 0x5
    exp = torch.from_numpy(orc.lower_median_cols(rows.float().cpu().numpy())).to(dtype)
    gu.assert_same(out.cpu(), exp, f"median {dtype} K={K} N={N}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [2, 3, 64, 127, 128, 129, 300, 512, 1100])
def test_median_signed_zero_ties_take_the_total_order(dtype, K, cuda_device):
    """Columns whose lower median falls among a mix of -0.0 and +0.0: every
    kernel family returns the zero of the IEEE total order (-0 < +0), which
    the oracle restates (torch's nth_element leaves that sign to the column's
    input order: DESIGN.md §5b, unpinned).  Columns vary the number of
    negatives, negative zeros and positive zeros around the rank, in both
    input orders, aligned (packed 16-bit kernels) and not."""
    N = 1_031
    g = torch.Generator().manual_seed(K)
    rows = torch.zeros(K, 1_088, dtype=torch.float32)
    for c in range(N):
        n_neg = int(torch.randint(0, K // 2 + 1, (1,), generator=g))
        n_nz = int(torch.randint(0, K - n_neg + 1, (1,), generator=g))
        col = torch.cat([-torch.rand(n_neg, generator=g) - 0.5, torch.full((n_nz,), -0.0),
                         torch.zeros(K - n_neg - n_nz), ])
        col[n_neg + n_nz:][: max(0, K - n_neg - n_nz - K // 3)] = torch.rand(max(0, K - n_neg - n_nz - K // 3),
                                                                             generator=g) + 0.5
        rows[:, c] = col[torch.randperm(K, generator=g)] if c % 2 else col.flip(0)
    rows = rows.to(dtype).to(cuda_device)[:, :N]
    d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(K)], cuda_device)
    out = torch.empty(1_088, dtype=dtype, device=cuda_device)[:N]
    dfn.median_rows(d_ptrs, K, N, out, aligned=True)
    exp = torch.from_numpy(orc.lower_median_cols(rows.float().cpu().numpy())).to(dtype)
    zeros = int((exp == 0).sum())
    assert zeros > N // 10, zeros  # the case exercises the ties
    gu.assert_same(out.cpu(), exp, f"median {dtype} K={K}")
