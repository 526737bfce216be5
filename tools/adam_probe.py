"""Time tile shapes of the fp32 reduction kernel at config 5 for its three
epilogues (plain FedAvg, fused server SGD+momentum, fused server Adam); tool
only.  Writes gpurun_out/adam_probe.json.  Variants interleaved in one
process, medians reported; not a parity check (tests/test_gpu_fedopt.py is)."""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libadam_probe.so")
sys.path.insert(0, os.path.dirname(HERE))
NV = 7
EPIS = {"fedavg": (0, 1), "sgd": (1, 4), "adam": (2, 6)}  # kind, extra N-sized fp32 streams


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "adam_probe.hip")
    deps = [src, os.path.join(HERE, "..", "fedml_amd", "csrc", "fedagg.hip")]
    if not os.path.exists(SO) or max(os.path.getmtime(d) for d in deps) > os.path.getmtime(SO):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-gpu-flush-denormals-to-zero", "-fPIC", "-shared", "-o", SO, src], check=True)
    return SO


def main():
    build()
    from fedml_amd import kernels as kn

    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.adam_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int64, P, P, P, P, ctypes.c_int, P]
    lib.adam_probe_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    K, N = 64, 4_194_304
    rows = torch.randn((K, N), device=dev) * 0.05
    tab = kn.upload_i64([rows[i].data_ptr() for i in range(K)], dev)
    p = torch.randn(N, device=dev)
    m = torch.zeros(N, device=dev)
    v = torch.zeros(N, device=dev)
    w = (ctypes.c_float * K)(*([1.0 / K] * K))
    sc = kn.adam_scalars(1.0, 0.9, 0.999, 1e-8, 2)
    st = torch.cuda.current_stream().cuda_stream
    names = [lib.adam_probe_name(i).decode() for i in range(NV)]
    res = {(e, n): [] for e in EPIS for n in names}

    def go(i, kind):
        rc = lib.adam_probe_launch(i, kind, tab.data_ptr(), w, K, N, p.data_ptr(), m.data_ptr(), v.data_ptr(),
                                   ctypes.addressof(sc), 0, st)
        assert rc == 0, rc

    for e, (kind, _) in EPIS.items():
        for i in range(NV):
            go(i, kind)
    torch.cuda.synchronize()
    reps = 20
    for _ in range(5):
        for e, (kind, _) in EPIS.items():
            for i in range(NV):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    go(i, kind)
                e1.record()
                torch.cuda.synchronize()
                res[(e, names[i])].append(e0.elapsed_time(e1) / reps)
    out = {}
    for (e, n), t in res.items():
        nbytes = K * N * 4 + EPIS[e][1] * N * 4
        ms = statistics.median(t)
        out.setdefault(e, {})[n] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}
    print(json.dumps(out, indent=1))
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/adam_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
