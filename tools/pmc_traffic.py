"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

    python tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch/bench_counter_collection.csv \
        --write gpurun_out/pmc_write/bench_counter_collection.csv --key cfg3:single \
        --kernel OpF32 --alg-bytes 13214838432

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly
half of the bytes of a wide (16 B/lane) coalesced streaming read, so the read
side is FETCH_SIZE x 2; WRITE_SIZE is exact for 16-byte streaming stores.
Both counters are in KiB.  The two counters come from separate passes (they
do not fit one TCC pass).  Results are merged into profiles/pmc_traffic.json,
which bench.py reads for its roofline.traffic field.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path: str, counter: str, kernel: str):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel {kernel!r} in {path}")
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--kernel", default="OpF32")
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch_kib, nf = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    write_kib, nw = per_launch(a.write, "WRITE_SIZE", a.kernel)
    read_b = 2 * fetch_kib * 1024
    write_b = write_kib * 1024
    rec = {
        "bytes_per_launch": int(round(read_b + write_b)),
        "read_bytes": int(round(read_b)),
        "write_bytes": int(round(write_b)),
        "FETCH_SIZE_KiB": fetch_kib,
        "WRITE_SIZE_KiB": write_kib,
        "launches_sampled": [nf, nw],
        "alg_bytes_per_launch": a.alg_bytes,
        "traffic_over_alg": round((read_b + write_b) / a.alg_bytes, 5),
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count for 16-B/lane streams), write = WRITE_SIZE; KiB",
    }
    try:
        allrec = json.load(open(a.out))
    except (OSError, ValueError):
        allrec = {}
    allrec[a.key] = rec
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(allrec, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({a.key: rec}, indent=1))


if __name__ == "__main__":
    main()
