"""bench.py's committed measurement tables (CPU): the PMC traffic table and the
median VALU table it reads load, key the way bench.py looks them up, and the
median's VALU-issue fraction is computed from them as documented
(DESIGN.md §5b)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_median_valu_table_keys_and_fields():
    d = json.load(open(os.path.join(ROOT, "profiles", "median_valu.json")))
    for key in ("cfg3:single:median", "cfg4:single:median", "cfg4:single:median@K512"):
        assert key in d, key
        e = d[key]
        assert e["valu_instr_per_wave"] > 100 and e["waves_per_launch"] > 1000
    assert bench.load_median_valu("cfg4", "single", 1, "median@K512") == d["cfg4:single:median@K512"]
    assert bench.load_median_valu("cfg4", "single", 1, "median@K7") is None


def test_median_valu_issue_fraction_formula():
    e = bench.load_median_valu("cfg4", "single", 1, "median@K512")
    issue_ms = e["valu_instr_per_wave"] * e["waves_per_launch"] * bench.VALU_HALF_RATE_CYCLES / (
        bench.SIMDS * bench.CLOCK_GHZ * 1e9) * 1e3
    # one wave64 half-rate instruction per 4 cycles per SIMD, 1,024 SIMDs at 2.4 GHz
    assert bench.SIMDS == 1024 and bench.VALU_HALF_RATE_CYCLES == 4
    assert 15.0 < issue_ms < 30.0  # config 4 at 512 clients: ~5,300 instructions x 2.7M waves


def test_traffic_table_keys():
    assert bench.load_traffic("cfg3", "single", 1) is not None
    assert bench.load_traffic("cfg3", "client", 8) is None or isinstance(bench.load_traffic("cfg3", "client", 8), int)
