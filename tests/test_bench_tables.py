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
    for key in ("cfg3:single:median@K128", "cfg4:single:median@K128", "cfg4:single:median@K512"):
        assert key in d, key
        e = d[key]
        assert e["valu_instr_per_wave"] > 100 and e["waves_per_launch"] > 1000
    assert bench.load_median_valu("cfg4", "single", 1, "median", 512) == d["cfg4:single:median@K512"]
    assert bench.load_median_valu("cfg4", "single", 1, "median", 7) is None


def test_median_valu_issue_fraction_formula():
    e = bench.load_median_valu("cfg4", "single", 1, "median", 512)
    issue_ms = e["valu_instr_per_wave"] * e["waves_per_launch"] * bench.VALU_HALF_RATE_CYCLES / (
        bench.SIMDS * bench.CLOCK_GHZ * 1e9) * 1e3
    # one wave64 half-rate instruction per 4 cycles per SIMD, 1,024 SIMDs at 2.4 GHz
    assert bench.SIMDS == 1024 and bench.VALU_HALF_RATE_CYCLES == 4
    # config 4 at 512 clients, the streamed bit-plane select (round 6): ~2.45M instructions per
    # persistent wave x 1,026 waves = ~4.1 ms of issue in a ~15-ms kernel (the counting kernel
    # before it: 3,619 x 2.7M waves = 16.3 ms in 21.3)
    assert 3.0 < issue_ms < 8.0


def test_traffic_table_keys():
    assert bench.load_traffic("cfg3", "single", 1, "", 128) is not None
    assert bench.load_traffic("cfg3", "single", 1, "", 7) is None
    assert bench.table_key("cfg4", "param", 4, "", 512) == "cfg4:param@K512"
    assert bench.table_key("cfg4", "param", 1, "median", 512) == "cfg4:single:median@K512"
    v = bench.load_traffic("cfg3", "client", 8, "", 16)
    assert v is None or isinstance(v, int)


def _baseline_clients():
    """The client count each BASELINE.json config names ("... 512 clients x ...")."""
    import re

    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    return [int(re.search(r"(\d+) clients", c).group(1)) for c in cfgs]


def test_bench_configs_keep_baseline_client_counts():
    """Every bench config aggregates BASELINE's clients: 4 / 32 / 128 / 512 / 64,
    at one GPU and over N GPUs in both partitionings (the client axis deals
    them out, the parameter axis gives every rank all of them)."""
    ks = _baseline_clients()
    assert ks == [4, 32, 128, 512, 64]
    for i, k in enumerate(ks):
        name = f"cfg{i + 1}"
        assert bench.CONFIGS[name]["K"] == k
        assert bench.plan_clients(name, 1, 0, "single") == (k, k, 0)
        for world in (2, 4, 8):
            for r in range(world):
                assert bench.plan_clients(name, world, r, "param") == (k, k, 0)
            if k < world:
                continue
            plans = [bench.plan_clients(name, world, r, "client") for r in range(world)]
            assert all(p[0] == k for p in plans)
            assert sum(p[1] for p in plans) == k
            assert [p[2] for p in plans] == [sum(q[1] for q in plans[:r]) for r in range(world)]


def test_bench_argv_cfg4_four_gpus_is_512_clients():
    """`bench.py --config cfg4 --gpus 4` (config 4's own deployment) parses to
    512 clients in both modes, 128 per GPU on the client axis."""
    a = bench.parse(["--config", "cfg4", "--gpus", "4"])
    assert a.mode == "param" and not a.no_exchange
    assert bench.plan_clients(a.config, 4, 3, "param", a.clients_total, a.weak, a.clients) == (512, 512, 0)
    a = bench.parse(["--config", "cfg4", "--gpus", "4", "--mode", "client"])
    assert bench.plan_clients(a.config, 4, 3, "client", a.clients_total, a.weak, a.clients) == (512, 128, 384)
    a = bench.parse(["--config", "cfg3", "--gpus", "8", "--weak"])
    assert bench.plan_clients(a.config, 8, 7, "client", a.clients_total, a.weak, a.clients) == (1024, 128, 896)
