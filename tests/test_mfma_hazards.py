"""MFMA -> VALU wait states of the shipped Gram kernels, read from the code
object (CPU: llvm-objdump + a data-flow over each kernel's control flow,
tools/mfma_hazards.py).

The round-4 compile left only 3 wait states between the last MFMA of the
Gram's accumulation chain and the fp64 fold on one path (10 % wrong distances
on the box at K <= 16); the fold now sits behind `s_nop 15` guards in
csrc/robust.hip.  These tests pin that in the binary that ships, and prove the
check would catch a removed guard by compiling robust.hip without them.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

from tools import mfma_hazards as mh
from tools.kernel_resources import LIB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "fedml_amd", "csrc", "robust.hip")
GUARD = re.compile(r'asm volatile\("s_nop 15" : "\+v"\(acc\[j\]\)\);')


@pytest.fixture(scope="module")
def shipped():
    if not os.path.exists(LIB):
        pytest.skip("libfedagg.so not built")
    return mh.check(LIB)


def test_every_gram_kernel_is_checked(shipped):
    gram = [k for k in shipped if "pairgram_split8_kernel" in k]
    assert len(gram) == 8, sorted(shipped)  # NB = 1 .. 8


def test_shipped_mfma_consumers_are_padded(shipped):
    bad = {k: v for k, v in shipped.items() if v}
    assert not bad, bad


def test_guards_in_source():
    assert len(GUARD.findall(open(SRC).read())) >= 1


def test_check_catches_a_removed_guard(tmp_path):
    """robust.hip with every guard deleted, device code only (~10 s): where the
    fold reads the MFMA accumulators directly (NB = 1, 2, 3, 8 in this
    compile; NB = 1 is the round-4 failure) it then gets only the compiler's
    own padding (8 states, or fewer as in round 4), below the 16 the guards
    promise.  (NB = 4..7 copy the accumulators with v_mov_b64 after a full
    s_nop 7 first and fold the copies, which needs no guard.)"""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = open(SRC).read()
    stripped, n = GUARD.subn(";", src)
    assert n >= 1
    d = tmp_path / "a" / "b"
    d.mkdir(parents=True)
    (tmp_path / "include").symlink_to(os.path.join(ROOT, "include"))
    (d / "robust.hip").write_text(stripped)
    obj = tmp_path / "robust_noguard.o"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt",
                    "--cuda-device-only", "-c", "-o", str(obj), str(d / "robust.hip")], check=True, timeout=600)
    res = mh.check(str(obj))
    gram = {k: v for k, v in res.items() if "pairgram_split8_kernel" in k}
    assert len(gram) == 8
    flagged = [k for k, v in gram.items() if v]
    assert any("ILi1E" in k for k in flagged) and len(flagged) >= 3, {k: len(v) for k, v in gram.items()}
    assert all("v_cvt_f64_f32" in x for v in gram.values() for x in v)
