"""bench.py's multi-rank orchestration on the CPU:
`--probe-cpu` runs the real coordination (host-store barriers and timing
gathers, the readiness handshake, the budget, the watchdog, the nested legs
and the JSON line) with host stand-in reductions over gloo, and the
FEDAGG_BENCH_FAIL / FEDAGG_BENCH_HANG hooks break one rank on purpose."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FEDAGG_BENCH_FAIL", "FEDAGG_BENCH_HANG"):
        e.pop(k, None)
    e.update(env or {})
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--probe-cpu", "--backend", "gloo",
                        "--steps", "3", "--warmup", "1"] + args, capture_output=True, text=True, timeout=timeout,
                       env=e, cwd=ROOT)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p, lines, time.monotonic() - t0


def test_all_legs_run_and_one_line_is_printed():
    p, lines, _ = _run(["--gpus", "2", "--nest", "cfg4,cfg5"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 2 and line["value"] > 0 and "probe" in line
    for obj in (line["exchange"], line["inprocess"], line["cfg4"]["param"], line["cfg4"]["exchange"],
                line["cfg4"]["inprocess"], line["cfg5"]["sharded_fedopt"], line["cfg5"]["inprocess_fedopt"]):
        assert "error" not in obj and "skipped" not in obj, obj
        assert obj["ms_per_step"] > 0
    assert line["exchange"]["backend"] == "gloo"


def test_a_rank_failing_in_the_exchange_leg_costs_only_that_leg():
    """Rank 1 fails after setup, before the collective: both ranks skip the
    collective, rank 0 still prints the headline with exchange.error, rc 0,
    well within a minute; the legs after it still run."""
    p, lines, took = _run(["--gpus", "2"], env={"FEDAGG_BENCH_FAIL": "exchange:1"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert took < 60
    assert len(lines) == 1
    line = lines[0]
    assert line["value"] > 0
    err = line["exchange"]["error"]
    assert "rank 1" in err and "injected failure" in err
    assert "error" not in line["inprocess"]


def test_a_rank_failing_in_a_nested_config_leg():
    p, lines, _ = _run(["--gpus", "2", "--nest", "cfg4"], env={"FEDAGG_BENCH_FAIL": "cfg4/exchange:0"})
    assert p.returncode == 0, p.stderr[-3000:]
    line = lines[0]
    assert "injected failure" in line["cfg4"]["exchange"]["error"]
    assert "error" not in line["cfg4"]["param"] and "error" not in line["cfg4"]["inprocess"]


def test_budget_skips_nested_legs_instead_of_overrunning():
    p, lines, _ = _run(["--gpus", "2", "--nest", "cfg4", "--budget-s", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    line = lines[0]
    assert line["value"] > 0
    for obj in (line["exchange"], line["inprocess"], line["cfg4"]["param"]):
        assert obj["skipped"].startswith("budget"), obj


def test_watchdog_prints_the_line_when_a_collective_never_returns():
    """Rank 1 hangs after the handshake, so rank 0 waits inside gloo's
    reduce-scatter: the watchdog prints the line with the headline and ends
    every rank with rc 0, long before the process group's 120 s timeout."""
    p, lines, took = _run(["--gpus", "2", "--watchdog-s", "25"], env={"FEDAGG_BENCH_HANG": "exchange:1"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert took < 60
    assert len(lines) == 1
    line = lines[0]
    assert line["value"] > 0 and "exchange" in line["watchdog"]
