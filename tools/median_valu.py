"""Executed VALU instructions per wave of the shipped median kernels (tool only).

    python tools/median_valu.py collect   # on the GPU box: one SQ pass per bench shape
    python tools/median_valu.py merge     # parse the passes into profiles/median_valu.json

Each pass is `rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace` over
`bench.py --op median` at one shape; instructions per wave = sum of
SQ_INSTS_VALU / sum of SQ_WAVES over the median kernel's launches.  bench.py
reads the table to report the median's VALU roofline: the sorting networks'
min / max / med3 / DPP ops issue at 4 cycles per wave64 instruction per SIMD
(tools/valu_rate_probe.hip), so instructions x 4 cycles over the kernel time
is the fraction of the SIMDs' issue capacity the kernel uses.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT_DIR = os.path.join(ROOT, "gpurun_out", "median_valu")
SHAPES = {  # key (as bench.py's load_traffic) -> bench.py arguments
    "cfg3:single:median@K128": ["--config", "cfg3"],
    "cfg4:single:median@K128": ["--config", "cfg4", "--clients", "128"],
    "cfg4:single:median@K512": ["--config", "cfg4"],
    "cfg3:single:median@K512": ["--config", "cfg3", "--clients", "512"],
}


def collect():
    os.makedirs(OUT_DIR, exist_ok=True)
    for key, args in SHAPES.items():
        d = os.path.join(OUT_DIR, key.replace(":", "_").replace("@", "_"))
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", "SQ_INSTS_VALU", "SQ_WAVES", "--kernel-trace",
               "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable, os.path.join(ROOT, "bench.py"),
               "--op", "median", *args, "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
        with open(d + ".log", "w") as log:
            rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT).returncode
        if rc != 0:
            raise SystemExit(f"{key}: rocprofv3 exited {rc} (see {d}.log)")
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            if "counter_collection" not in f and os.path.getsize(f) > 1 << 20:
                os.remove(f)


def merge():
    res = {}
    for key in SHAPES:
        d = os.path.join(OUT_DIR, key.replace(":", "_").replace("@", "_"))
        files = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
        if not files:
            continue
        sums, names, launches = {"SQ_INSTS_VALU": 0.0, "SQ_WAVES": 0.0}, set(), set()
        for r in csv.DictReader(open(files[0])):
            if "median" not in r["Kernel_Name"]:
                continue
            sums[r["Counter_Name"]] += float(r["Counter_Value"])
            m = re.search(r"(median_\w+<[^()]*>)", r["Kernel_Name"])
            names.add(m.group(1) if m else r["Kernel_Name"][:120])
            launches.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        if sums["SQ_WAVES"]:
            res[key] = {"valu_instr_per_wave": round(sums["SQ_INSTS_VALU"] / sums["SQ_WAVES"], 1),
                        "waves_per_launch": round(sums["SQ_WAVES"] / max(1, len(launches))),
                        "kernels": sorted(names), "launches_sampled": len(launches),
                        "counters": "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES, summed over the median launches"}
    path = os.path.join(ROOT, "profiles", "median_valu.json")
    json.dump(res, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"collect": collect, "merge": merge}[sys.argv[1]]()
