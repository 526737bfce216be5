"""CPU-side checks of the boundary: the library loads, exports every symbol the
header declares with the ctypes signatures we bind, validates arguments
without touching a GPU, and the product path refuses to run without one."""
from __future__ import annotations

import os
import re
from collections import OrderedDict

import pytest
import torch

from fedml_amd import _native as nat
from fedml_amd import build as fbuild

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fedagg.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fedagg_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    fbuild.build()
    return nat.lib()


def test_every_header_symbol_exported(lib):
    names = header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(nat.SIGNATURES), "ctypes signatures out of sync with include/fedagg.h"


def test_product_library_exports_only_the_drop_in_abi(lib):
    """libfedagg.so's dynamic symbol table holds exactly include/fedagg.h's
    functions (plus the compiler's __hip_cuid markers): no tuning entries,
    no internal helpers or globals."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", fbuild.OUT], capture_output=True, text=True,
                         check=True).stdout
    exported = set()
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3 and parts[1] in "TDBR" and not parts[2].startswith("__hip_cuid"):
            exported.add(parts[2])
    assert exported == set(header_functions()), sorted(exported ^ set(header_functions()))


def test_library_is_gfx950_code_object():
    path = fbuild.build()
    data = open(path, "rb").read()
    assert b"gfx950" in data
    assert b"__hip_fatbin" in data or b"HIP_FATBIN" in data or b".hip_fatbin" in data


def test_argument_validation_without_gpu(lib):
    # invalid sizes are rejected before any HIP call
    assert lib.fedagg_wsum_f32(None, None, 0, 10, None, 0, None) == -1
    assert b"K must be" in lib.fedagg_last_error()
    assert lib.fedagg_wsum_f32(None, None, 4, -1, None, 0, None) == -1
    assert lib.fedagg_wsum_bf16(1, 1, 2, 10, 1, 7, 1, None) == -1
    assert lib.fedagg_sum(99, 1, 2, 10, 1, 0, None) == -1
    assert lib.fedagg_multi_blocks(nat.DT_F64, 100) == -1
    assert lib.fedagg_multi_blocks(nat.DT_F32, -1) == -1
    assert lib.fedagg_wsum_multi(nat.DT_F64, 0, 1, 1, 1, 1, 1, 1, 2, 1, None) == -1
    assert lib.fedagg_wsum_multi(nat.DT_BF16, 5, 1, 1, 1, 1, 1, 1, 2, 1, None) == -1
    assert lib.fedagg_wsum_multi(nat.DT_F32, 0, None, 1, 1, 1, 1, 1, 2, 1, None) == -1
    assert lib.fedagg_version() == 1
    assert lib.fedagg_device_round_f32(None, None, None, 0, 1, None, None, None) == -1
    assert lib.fedagg_wsum_fedopt_optrepo_f32(9, 1, 1, 1, 1, 1, 1, 1, 1, 0, None) == -1


def test_multi_block_plan(lib):
    from fedml_amd.kernels import MultiF32Plan

    plan = MultiF32Plan([0, 1, 4096, 25_000_000])
    assert plan.block_begin[0] == 0 and plan.block_begin[1] == 0
    assert plan.block_begin[2] == 1
    per_block = 4096 // (plan.block_begin[3] - plan.block_begin[2])
    assert per_block >= 1024
    assert plan.total_blocks == plan.block_begin[-1]


@pytest.mark.parametrize("dtype,elems_per_block", [(torch.float32, 4096), (torch.bfloat16, 8192),
                                                     (torch.float16, 8192), (torch.int64, 2048)])
def test_multi_plan_dtypes(lib, dtype, elems_per_block):
    from fedml_amd.kernels import MultiPlan

    plan = MultiPlan([0, 1, elems_per_block, elems_per_block + 1, 10 * elems_per_block], dtype)
    assert plan.block_begin == [0, 0, 1, 2, 4, 14]
    with pytest.raises(TypeError):
        MultiPlan([1], torch.float64)


def test_no_cpu_fallback():
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    from fedml_amd.agg_operator import FedMLAggOperator

    raw = [(1, OrderedDict(a=torch.ones(3))), (3, OrderedDict(a=torch.zeros(3)))]
    with pytest.raises(nat.FedAggNativeError):
        FedMLAggOperator.agg(type("A", (), {"federated_optimizer": "FedAvg"})(), raw)


def test_reference_errors_before_device_work():
    """Errors the reference raises on the host come out identically, without a GPU."""
    from fedml_amd.agg_operator import FedMLAggOperator

    A = type("A", (), {"federated_optimizer": "FedAvg"})
    with pytest.raises(ZeroDivisionError):
        FedMLAggOperator.agg(A(), [(0, OrderedDict(a=torch.ones(3))), (0, OrderedDict(a=torch.ones(3)))])
    with pytest.raises(ValueError):
        FedMLAggOperator.agg(A(), [(1, OrderedDict(a=torch.ones(3)), OrderedDict())])
    with pytest.raises(UnboundLocalError):
        FedMLAggOperator.agg(type("B", (), {"federated_optimizer": "FedOpt"})(), [(1, OrderedDict())])
    with pytest.raises(NotImplementedError):
        FedMLAggOperator.agg(type("C", (), {"federated_optimizer": "FedAvg", "ml_engine": "tf"})(),
                             [(1, OrderedDict())])
    # empty state dict: the reference never divides, returns client 0's dict
    d = OrderedDict()
    assert FedMLAggOperator.agg(A(), [(0, d)]) is d


def test_server_aggregator_surface():
    from fedml_amd.server_aggregator import MI355XServerAggregator

    m = torch.nn.Linear(3, 2)
    args = type("A", (), {"federated_optimizer": "FedAvg"})()
    agg = MI355XServerAggregator(m, args)
    sd = agg.get_model_params()
    assert list(sd.keys()) == ["weight", "bias"]
    lst = [(1, sd), (2, sd)]
    out, idxs = agg.on_before_aggregation(lst)
    assert out is lst and idxs == [0, 1]
    x = OrderedDict(a=torch.ones(1))
    assert agg.on_after_aggregation(x) is x
    with pytest.raises(NotImplementedError):
        MI355XServerAggregator(m, type("B", (), {"federated_optimizer": "FedAvg", "enable_dp": True})())


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_host_pack_gathers_exactly(lib, threads):
    """fedagg_host_pack is host code: check it fully on CPU (ragged sizes, gaps,
    sizes above the threading threshold)."""
    import ctypes

    import numpy as np

    rng = np.random.default_rng(0)
    sizes = [0, 1, 7, 4096, 3_000_001, 5, 2_500_000]
    srcs = [rng.integers(0, 255, s, dtype=np.uint8) for s in sizes]
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += s + 3  # gaps stay untouched
    dst = np.full(o, 0xAB, dtype=np.uint8)
    n = len(sizes)
    rc = lib.fedagg_host_pack(dst.ctypes.data, (ctypes.c_void_p * n)(*[a.ctypes.data for a in srcs]),
                              (ctypes.c_int64 * n)(*offs), (ctypes.c_int64 * n)(*sizes), n, threads)
    assert rc == 0
    for a, off in zip(srcs, offs):
        assert np.array_equal(dst[off:off + a.size], a)
        assert dst[off + a.size] == 0xAB
    assert lib.fedagg_host_pack(None, None, None, None, -1, 1) == -1


def test_host_unpack_scatters_exactly(lib):
    import ctypes

    import numpy as np

    rng = np.random.default_rng(1)
    sizes = [3, 0, 5_000_003, 64, 1]
    src = rng.integers(0, 255, sum(sizes) + 40, dtype=np.uint8)
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += s + 8
    dsts = [np.zeros(s, dtype=np.uint8) for s in sizes]
    n = len(sizes)
    assert lib.fedagg_host_unpack(src.ctypes.data, (ctypes.c_void_p * n)(*[d.ctypes.data for d in dsts]),
                                  (ctypes.c_int64 * n)(*offs), (ctypes.c_int64 * n)(*sizes), n, 8) == 0
    for d, off in zip(dsts, offs):
        assert np.array_equal(d, src[off:off + d.size])


@pytest.mark.parametrize("threads", [1, 8, 16])
def test_host_gather_to_many_destinations(lib, threads):
    """fedagg_host_gather (the multi-device ingest's one pack for every GPU's
    staging row): each source lands in its own destination buffer, bytes
    around the destinations untouched, sizes above the threading threshold;
    several callers at once (the pack pool serves concurrent batches)."""
    import ctypes
    import threading

    import numpy as np

    rng = np.random.default_rng(2)
    sizes = [0, 9, 4_000_001, 3, 6_500_000, 1, 131_072]

    def one(seed):
        r = np.random.default_rng(seed)
        srcs = [r.integers(0, 255, s, dtype=np.uint8) for s in sizes]
        bufs = [np.full(s + 2, 0xCD, dtype=np.uint8) for s in sizes]  # one guard byte each side
        n = len(sizes)
        rc = lib.fedagg_host_gather((ctypes.c_void_p * n)(*[b.ctypes.data + 1 for b in bufs]),
                                    (ctypes.c_void_p * n)(*[a.ctypes.data for a in srcs]),
                                    (ctypes.c_int64 * n)(*sizes), n, threads)
        assert rc == 0
        for a, b in zip(srcs, bufs):
            assert np.array_equal(b[1:1 + a.size], a) and b[0] == 0xCD and b[-1] == 0xCD

    one(int(rng.integers(1 << 30)))
    errs = []

    def run(seed):
        try:
            one(seed)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ths = [threading.Thread(target=run, args=(s,)) for s in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs
    assert lib.fedagg_host_gather(None, None, None, -1, 1) == -1
    one_byte = np.zeros(1, dtype=np.uint8)
    assert lib.fedagg_host_gather((ctypes.c_void_p * 1)(None), (ctypes.c_void_p * 1)(one_byte.ctypes.data),
                                  (ctypes.c_int64 * 1)(1), 1, 1) == -1


def test_dict_walker_builds_and_declines_host_inputs():
    """The native dict walker (csrc/walker.cpp) only ever takes the all-device
    fast path; host tensors and missing keys return None so the Python walk
    handles them (and raises the reference's KeyError)."""
    from fedml_amd import agg_operator as ao

    w = ao._walker()
    assert w is not None, "build the walker: python -m fedml_amd.build"
    assert w.walk([OrderedDict(a=torch.ones(3))], ["a"]) is None
    assert w.walk([OrderedDict(a=torch.ones(3))], ["b"]) is None
    assert w.walk([], ["a"]) is None
    assert w.walk([OrderedDict(a=1)], ["a"]) is None

    class Custom(dict):
        def __getitem__(self, k):  # overridden lookup: never walked natively
            return super().__getitem__(k)

    assert w.walk([Custom(a=torch.ones(3))], ["a"]) is None
    assert w.walk([OrderedDict(a=torch.ones(3).to_sparse())], ["a"]) is None  # non-strided: no C++ throw escapes
    with pytest.raises(TypeError):
        w.walk([OrderedDict()], [["unhashable"]])


def test_dict_walker_order_by_size():
    """order_by_size: key indices largest tensor first, ties in key order;
    None where the walk would decline (missing key, non-tensor, custom dict)."""
    from fedml_amd import agg_operator as ao

    w = ao._walker()
    d = OrderedDict(a=torch.ones(3), b=torch.ones(10), c=torch.ones(3), d=torch.ones(()), e=torch.ones(2, 5))
    assert w.order_by_size(d, list(d)) == [1, 4, 0, 2, 3]
    assert w.order_by_size(d, ["a", "zz"]) is None
    assert w.order_by_size(OrderedDict(a=1), ["a"]) is None

    class Custom(dict):
        def __getitem__(self, k):
            return super().__getitem__(k)

    assert w.order_by_size(Custom(a=torch.ones(3)), ["a"]) is None
    assert w.walk([d], list(d), True) is None  # host tensors: declined before allocating
    chunks = [list(c) for c in ao._chunks(list(range(300)))]
    assert [len(c) for c in chunks[:len(ao._CHUNK_KEYS)]] == list(ao._CHUNK_KEYS)
    assert sum(chunks, []) == list(range(300)) and all(len(c) <= 96 for c in chunks[len(ao._CHUNK_KEYS):])


def test_dict_walker_pool_under_repeated_walks():
    """Walks of >= 4096 tensors validate on the walker's thread pool: repeated
    back-to-back walks finish (no lost wake-up or stale worker) and decline
    host tensors every time; subclass values (nn.Parameter) are declined
    before any validation thread sees them."""
    from fedml_amd import agg_operator as ao

    w = ao._walker()
    keys = [f"k{t}" for t in range(64)]
    dicts = [OrderedDict((k, torch.zeros(2)) for k in keys) for _ in range(128)]
    for _ in range(300):
        assert w.walk(dicts, keys) is None
        assert w.walk(dicts, keys[:8], True) is None  # below the pool threshold
    dicts[5][keys[3]] = torch.nn.Parameter(torch.zeros(2))
    assert w.walk(dicts, keys) is None



@pytest.mark.parametrize("K", [1, 3, 4, 129])
def test_weights_ride_in_pointer_table(K):
    """The device-dict path appends the fp32 weights to the first pointer
    table's upload: K floats, RNE from the Python floats as torch.tensor
    rounds them, two per int64 slot, zero-padded to an even count."""
    import numpy as np

    from fedml_amd import kernels as kn

    ns = [float(v) for v in np.random.default_rng(K).integers(1, 1000, K)]
    ws = [n / sum(ns) for n in ns]
    packed = kn.weights_as_i64(ws)
    assert packed.dtype == np.int64 and packed.size == (K + 1) // 2
    back = packed.view(np.float32)
    assert torch.equal(torch.from_numpy(back[:K].copy()), torch.tensor(ws, dtype=torch.float32))
    assert back.size == K or back[K] == 0.0


def test_fedopt_launch_struct_matches_the_header(tmp_path):
    """fedagg_fedopt_launch: the ctypes mirror (_native.FedOptLaunch) has the
    C struct's size and field offsets (compiled against include/fedagg.h)."""
    import ctypes
    import shutil
    import subprocess

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    fields = [f for f, _ in nat.FedOptLaunch._fields_]
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "fedagg.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(fedagg_fedopt_launch));\n' +
                   "".join(f'  printf("%zu\\n", offsetof(fedagg_fedopt_launch, {f}));\n' for f in fields) +
                   "  return 0;\n}\n")
    exe = tmp_path / "sz"
    subprocess.run([cc, "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got[0] == ctypes.sizeof(nat.FedOptLaunch)
    assert got[1:] == [getattr(nat.FedOptLaunch, f).offset for f in fields]


def test_fedopt_batch_validation_without_gpu(lib):
    assert lib.fedagg_wsum_fedopt_batch(None, 0) == 0  # nothing to launch
    assert lib.fedagg_wsum_fedopt_batch(None, 2) == -1
