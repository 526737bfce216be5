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
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "fedagg.hip")
# every translation unit of libfedagg.so: compiled to objects separately (an
# unchanged unit is not recompiled), then linked
SRCS = [SRC, os.path.join(HERE, "csrc", "robust.hip"), os.path.join(HERE, "csrc", "median.hip")]
OUT_DIR = os.path.join(HERE, "lib")
OBJ_DIR = os.path.join(OUT_DIR, "obj")
OUT = os.path.join(OUT_DIR, "libfedagg.so")
WALKER_SRC = os.path.join(HERE, "csrc", "walker.cpp")
WALKER_OUT = os.path.join(OUT_DIR, "_fedagg_walker" + sysconfig.get_config_var("EXT_SUFFIX"))
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
    "-Wall",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


HEADER = os.path.join(HERE, "..", "include", "fedagg.h")


def _obj(src: str) -> str:
    return os.path.join(OBJ_DIR, os.path.splitext(os.path.basename(src))[0] + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    return any(os.path.getmtime(d) > os.path.getmtime(target) for d in deps if os.path.exists(d))


def needs_rebuild() -> bool:
    return _stale(OUT, SRCS + [HEADER, __file__])


def build_walker(force: bool = False, verbose: bool = False) -> str:
    """The host-side dict walker (csrc/walker.cpp): a CPython module built
    against torch's headers with the system C++ compiler (no device code)."""
    if not force and os.path.exists(WALKER_OUT) and \
            os.path.getmtime(WALKER_OUT) >= max(os.path.getmtime(WALKER_SRC), os.path.getmtime(__file__)):
        return WALKER_OUT
    import torch
    from torch.utils import cpp_extension as ce

    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = WALKER_OUT + ".tmp"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I" + sysconfig.get_paths()["include"],
           *("-I" + d for d in ce.include_paths()), WALKER_SRC,
           *("-L" + d for d in ce.library_paths()), "-ltorch_python", "-ltorch", "-lc10",
           *("-Wl,-rpath," + d for d in ce.library_paths()), "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, WALKER_OUT)
    return WALKER_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_walker(force=force, verbose=verbose)
    if not force and not needs_rebuild():
        return OUT
    os.makedirs(OBJ_DIR, exist_ok=True)
    objs = [_obj(src) for src in SRCS]
    # the translation units compile side by side (one hipcc each)
    jobs = []
    for src, obj in zip(SRCS, objs):
        if force or _stale(obj, [src, HEADER, __file__]):
            tmp = obj + ".tmp.o"
            cmd = [hipcc(), *HIPCC_FLAGS, "-c", "-o", tmp, src]
            if verbose:
                print(" ".join(cmd))
            # each unit's diagnostics are collected apart, so a failure prints
            # one unit's errors instead of every hipcc's interleaved output
            jobs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), cmd, tmp, obj))
    failed = []
    for p, cmd, tmp, _ in jobs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((cmd, out))
        elif out and verbose:
            sys.stdout.write(out.decode(errors="replace"))
    if failed:
        for _, _, tmp, _ in jobs:  # no half-built objects left behind
            if os.path.exists(tmp):
                os.remove(tmp)
        cmd, out = failed[0]
        sys.stderr.write(out.decode(errors="replace"))
        raise subprocess.CalledProcessError(1, cmd, output=out)
    for _, _, tmp, obj in jobs:
        os.replace(tmp, obj)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
