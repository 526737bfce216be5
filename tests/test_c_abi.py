"""The C ABI from a C++ host program (no Python in the loop): build here, run
on the GPU, compare with the C oracle bit for bit (tests/c/abi_test.cpp)."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "abi_test.cpp")
ORACLE = os.path.join(ROOT, "oracle", "fedavg_oracle.c")
OUT_DIR = os.path.join(ROOT, "tests", "c", "_build")
BIN = os.path.join(OUT_DIR, "abi_test")


def build_abi_test() -> str:
    from fedml_amd import build as fbuild

    lib = fbuild.build()
    os.makedirs(OUT_DIR, exist_ok=True)
    deps = [SRC, ORACLE, lib]
    if os.path.exists(BIN) and all(os.path.getmtime(d) <= os.path.getmtime(BIN) for d in deps):
        return BIN
    obj = os.path.join(OUT_DIR, "oracle.o")
    subprocess.run(["gcc", "-O2", "-std=c11", "-fPIE", "-ffp-contract=off", "-c", ORACLE, "-o", obj], check=True)
    main_o = os.path.join(OUT_DIR, "abi_test.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIE", "-c", SRC, "-o", main_o], check=True)
    libdir = os.path.dirname(lib)
    subprocess.run(["g++", main_o, obj, "-o", BIN, "-L" + libdir, "-lfedagg", "-Wl,-rpath," + libdir,
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-lm"], check=True)
    return BIN


def test_abi_program_builds():
    assert os.path.exists(build_abi_test())


@pytest.mark.gpu
def test_abi_program_runs_on_gpu(cuda_device):
    r = subprocess.run([build_abi_test()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ABI OK" in r.stdout, r.stdout + r.stderr
