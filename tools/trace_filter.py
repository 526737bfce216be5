"""Keep the rows of a rocprofv3 kernel-trace CSV whose kernel name matches a
substring, with start/end times relative to the first kept row (a trace of a
run that also launches tens of thousands of setup kernels is too large to
bring back whole).

    python tools/trace_filter.py TRACE.csv SUBSTRING OUT.csv
"""
import csv
import sys


def main():
    src, pat, dst = sys.argv[1:4]
    rows = []
    with open(src, newline="") as f:
        for r in csv.DictReader(f):
            if pat in r["Kernel_Name"]:
                rows.append(r)
    if not rows:
        raise SystemExit(f"no kernel matches {pat!r}")
    t0 = int(rows[0]["Start_Timestamp"])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["start_us", "end_us", "dur_us", "grid", "kernel"])
        for r in rows:
            s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
            w.writerow([f"{s / 1e3:.1f}", f"{e / 1e3:.1f}", f"{(e - s) / 1e3:.1f}", r.get("Grid_Size_X", ""),
                        r["Kernel_Name"][:90]])


if __name__ == "__main__":
    main()
