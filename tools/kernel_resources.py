"""Resource usage of every kernel that SHIPS in fedml_amd/lib/libfedagg.so (tool only).

    python tools/kernel_resources.py [out.tsv]      # default profiles/r02/kernel_resources.tsv

Reads the gfx950 code object out of the library's offload bundle and its
AMDGPU metadata note (llvm-readelf --notes): per kernel the VGPR / AGPR / SGPR
counts, spills and scratch (private segment) bytes, and the occupancy those
VGPRs allow (512 unified registers per SIMD lane, 8-register granule,
8 waves max).  This is the record of what the build produced; rocprofv3's
kernel-trace VGPR_Count column is not the arch VGPR count on gfx950 (it read
40 for the headline kernel whose code object says 130).
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fedml_amd", "lib", "libfedagg.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(lib: str = LIB):
    """The gfx950 code object of EVERY offload bundle in the library (one per
    translation unit: fedagg.hip and robust.hip)."""
    data = open(lib, "rb").read()
    out = []
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode(errors="replace")
            p += tl
            if "gfx950" in triple:
                out.append(data[i + off:i + off + size])
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 24)
    if not out:
        raise SystemExit("no gfx950 code object in " + lib)
    return out


def kernels(co: bytes):
    path = "/tmp/_fedagg_gfx950.co"
    open(path, "wb").write(co)
    notes = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, check=True).stdout
    out = []
    for block in re.split(r"\n\s*- \.agpr_count:", notes)[1:]:
        block = ".agpr_count:" + block

        def g(key):
            m = re.search(r"\." + key + r":\s+(\S+)", block)
            return m.group(1) if m else ""

        out.append({k: g(k) for k in ("name", "agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count",
                                      "sgpr_spill_count", "private_segment_fixed_size", "group_segment_fixed_size",
                                      "max_flat_workgroup_size")})
    names = subprocess.run(["c++filt"], input="\n".join(k["name"] for k in out), capture_output=True,
                           text=True).stdout.split("\n")
    for k, d in zip(out, names):
        d = d.replace("(anonymous namespace)::", "")
        k["kernel"] = re.sub(r"\(.*$", "", d).replace("void ", "")
        # gfx950's metadata .vgpr_count is the unified file's count (arch VGPRs
        # rounded up, then the AGPRs): 423 for 256 arch + 167 AGPRs
        v, a = int(k["vgpr_count"] or 0), int(k["agpr_count"] or 0)
        regs = v if v > 256 or a == 0 else (v + 3) // 4 * 4 + a
        regs = (regs + 7) // 8 * 8
        k["occupancy"] = min(8, 512 // max(regs, 1))
    return out


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03", "kernel_resources.tsv")
    ks = sorted((k for co in code_objects() for k in kernels(co)), key=lambda k: k["kernel"])
    cols = ["kernel", "vgpr_count", "agpr_count", "occupancy", "sgpr_count", "vgpr_spill_count",
            "sgpr_spill_count", "private_segment_fixed_size", "group_segment_fixed_size"]
    with open(out, "w") as f:
        f.write("\t".join(cols) + "\n")
        for k in ks:
            f.write("\t".join(str(k[c]) for c in cols) + "\n")
    scratch = [k for k in ks if int(k["private_segment_fixed_size"] or 0) or int(k["vgpr_spill_count"] or 0)]
    sgpr = [k for k in ks if int(k["sgpr_spill_count"] or 0)]
    print(f"{len(ks)} kernels, {len(scratch)} with scratch or VGPR spills, {len(sgpr)} with SGPR spills "
          f"(SGPR spills go to VGPR lanes, not memory) -> {out}")
    for k in scratch:
        print(f"  {k['kernel']}: scratch {k['private_segment_fixed_size']} B/lane, {k['vgpr_spill_count']} VGPR spills")
    for k in sgpr:
        print(f"  {k['kernel']}: {k['sgpr_spill_count']} SGPR spills, {k['vgpr_count']} VGPRs")


if __name__ == "__main__":
    main()
