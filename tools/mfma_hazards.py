"""MFMA -> vector-consumer wait states in the SHIPPED gfx950 code (tool + CPU test).

    python tools/mfma_hazards.py [library-or-object]

An XDL MFMA writes its destination VGPRs several passes after it issues; a
VALU (or LDS / memory) instruction that reads or overwrites those registers
too early sees stale values.  gfx950's v_mfma_f32_16x16x32_bf16 (4 passes,
16 cycles) needs 4 + 3 + 1 = 8 wait states before such a consumer (LLVM's
gfx950 rule for an XDL write followed by a VALU read; the compiler pads to
exactly that).  On the round-4 Gram kernels the compiler once left only 3
before the fold of the fp32 accumulators into fp64, and NB = 1 returned wrong
distances on the box; the fold now passes each accumulator through an
`asm volatile("s_nop 15")` guard (csrc/robust.hip), i.e. at least 16 wait
states on every path.  Two rules are checked:

* every vector consumer of an MFMA result: >= REQUIRED[mnemonic] states;
* every fold (GUARDED consumers: v_cvt_f64_f32 of an MFMA result): >= 16,
  so removing a guard fails the check even where the compiler's own padding
  happens to meet the ISA rule.

This checker disassembles every gfx950 code object in the library
(llvm-objdump), builds each kernel's control-flow graph from the branch
targets, and runs a forward data-flow over it: per VGPR, the MINIMUM number of
wait states since an MFMA wrote it along any path (loops included; merges take
the minimum).  Every instruction counts one wait state, `s_nop N` counts N + 1
(a lower bound: multi-cycle instructions only add more).  A non-MFMA vector
instruction whose operands touch a register below the requirement is a
violation.  MFMAs reading their own accumulator (srcC) are the hardware's
dependent-chain case and are not consumers here.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
from typing import Dict, List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools.kernel_resources import LIB, code_objects  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
# wait states an XDL result needs before a vector consumer, by mnemonic
REQUIRED = {"v_mfma_f32_16x16x32_bf16": 8}
DEFAULT_REQUIRED = 20  # 16-pass MFMAs (the longest); none ship today
GUARDED = {"v_cvt_f64_f32_e32": 16}  # the fp64 fold behind the s_nop 15 guards
_CAP = 64  # distances saturate here (well above any requirement)

_LINE = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-fA-F]+)>")
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _vregs(text: str) -> List[int]:
    out: List[int] = []
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(co: bytes) -> Dict[str, List[Tuple[int, str, str]]]:
    """{kernel symbol: [(address, mnemonic, operands), ...]}"""
    path = "/tmp/_fedagg_hazard.co"
    with open(path, "wb") as f:
        f.write(co)
    txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", path], capture_output=True, text=True,
                         check=True).stdout
    kernels: Dict[str, List[Tuple[int, str, str]]] = {}
    cur = None
    for line in txt.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            kernels[cur] = []
            continue
        m = _LINE.match(line)
        if m and cur is not None:
            mn, ops, addr, tail = m.groups()
            kernels[cur].append((int(addr, 16), mn, ops + (" " + tail.strip() if "<" in tail else "")))
    return kernels


def _successors(insts, i, base: int, index: Dict[int, int]) -> List[int]:
    addr, mn, ops = insts[i]
    nxt = [i + 1] if i + 1 < len(insts) else []
    if mn == "s_endpgm" or mn.startswith("s_setpc") or mn.startswith("s_trap"):
        return []
    if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
        m = _TARGET.search(ops)
        tgt = [index[base + int(m.group(2), 16)]] if m and base + int(m.group(2), 16) in index else []
        return tgt if mn.startswith("s_branch") else tgt + nxt
    return nxt


def check_kernel(insts) -> List[str]:
    """Violations in one kernel (empty if every consumer is padded)."""
    if not any(mn.startswith("v_mfma") for _, mn, _ in insts):
        return []
    base = insts[0][0]
    index = {a: i for i, (a, _, _) in enumerate(insts)}
    succ = [_successors(insts, i, base, index) for i in range(len(insts))]
    # state before instruction i: {vgpr: (wait states since its MFMA write, required)}
    state: List[Dict[int, Tuple[int, int]] | None] = [None] * len(insts)
    state[0] = {}
    work = [0]
    bad = {}
    while work:
        i = work.pop()
        cur = dict(state[i])
        addr, mn, ops = insts[i]
        regs = _vregs(ops.split("<")[0])
        if mn.startswith("v_mfma"):
            dst = _vregs(ops.split(",")[0])
            need = REQUIRED.get(mn, DEFAULT_REQUIRED)
            for r in dst:
                cur[r] = (-1, need)  # the MFMA's own issue slot is not a wait state
        elif regs and (mn.startswith("v_") or mn.startswith("ds_") or mn.startswith("global_")
                       or mn.startswith("buffer_") or mn.startswith("flat_")):
            for r in regs:
                if r in cur:
                    need = max(cur[r][1], GUARDED.get(mn, 0))
                    if cur[r][0] < need:
                        bad[addr] = f"{mn} {ops.split('<')[0].strip()} at 0x{addr:x}: v{r} {cur[r][0]} of {need} states"
            if mn.startswith("v_") and ops:
                for r in _vregs(ops.split(",")[0]):  # a VALU write ends the MFMA's claim on its destination
                    cur.pop(r, None)
        step = 1
        if mn == "s_nop":
            step = int(ops.split()[0], 0) + 1
        out = {r: (min(d + step, _CAP), need) for r, (d, need) in cur.items() if d + step < _CAP}
        for j in succ[i]:
            old = state[j]
            if old is None:
                state[j] = out
                work.append(j)
                continue
            merged = dict(old)
            changed = False
            for r, (d, need) in out.items():
                if r not in merged or d < merged[r][0]:
                    merged[r] = (d, need)
                    changed = True
            if changed:
                state[j] = merged
                work.append(j)
    return list(bad.values())


def check(path: str = LIB) -> Dict[str, List[str]]:
    """{kernel: violations} over every MFMA kernel of every gfx950 code object."""
    out: Dict[str, List[str]] = {}
    for co in code_objects(path):
        for name, insts in disassemble(co).items():
            if any(mn.startswith("v_mfma") for _, mn, _ in insts):
                out[name] = check_kernel(insts)
    return out


def main() -> None:
    res = check(sys.argv[1] if len(sys.argv) > 1 else LIB)
    for k, v in res.items():
        print(f"{len(v):4d}  {k}")
        for x in v[:5]:
            print("      ", x)
    sys.exit(1 if any(res.values()) else 0)


if __name__ == "__main__":
    main()
