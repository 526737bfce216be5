"""In-tree build of libfedagg.so for gfx950 (``python -m fedml_amd.build``).

hipcc cross-compiles without a GPU, so this runs in the CPU container too.  The
output lands in fedml_amd/lib/ and travels to the GPU box with the repo
snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "fedagg.hip")
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libfedagg.so")
ARCH = os.environ.get("FEDAGG_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    # Two roundings per client (mul, then add) exactly like torch's eager
    # `p * w` / `acc += t`: never contract to FMA (bit-exact parity).
    "-ffp-contract=off",
    # torch's CPU kernels keep fp32 denormals; so do we.
    "-fno-gpu-flush-denormals-to-zero",
    # IEEE division and sqrt (server Adam step); the HIP default, stated here
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fPIC",
    "-shared",
    "-Wall",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def needs_rebuild() -> bool:
    if not os.path.exists(OUT):
        return True
    deps = [SRC, os.path.join(HERE, "..", "include", "fedagg.h"), __file__]
    return any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_rebuild():
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
