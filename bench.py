#!/usr/bin/env python
"""Headline benchmark: device-resident FedAvg aggregation on MI355X.

One step = one server aggregation round over client updates already resident
in HBM: host computes the weights w_i = n_i/Σn, and the weighted-sum kernels
reduce every client row (one launch per dtype group).

Default workload = BASELINE.json config 3: 128 clients x ResNet-50 state dict
(25,610,152 fp32 + 53 int64 elements per client), synthetic data generated
in HBM.

Every config keeps BASELINE.json's client count (4 / 32 / 128 / 512 / 64;
`plan_clients`).  With --gpus N (one process per GPU) the round keeps it too
(strong scaling, ``--clients-total``, default the config's K):

  --mode param (default)  every rank holds ITS KEYS of every client (whole
                          keys dealt to ranks by bytes, the same partition as
                          the in-process fedml_amd.multidev bucket) and
                          reduces them in the reference order: no exchange,
                          bit-exact with one GPU.  Nested legs follow (below).
  --mode client           every rank holds its K/N clients' whole updates,
                          computes an fp32 partial and joins one chunked RCCL
                          reduce-scatter (timed separately on the comm stream).
  --weak                  round 2's weak scaling: every rank gets the
                          config's K clients of its own.

    python bench.py                       # 1 GPU, default steps
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8
    python bench.py --gpus 8              # the same: bench.py spawns the 8 ranks itself

Nested legs of a multi-GPU --mode param FedAvg line (each its own JSON object):

  exchange      north_star's client axis on the same clients: fp32 partials +
                the chunked RCCL reduce-scatter over xGMI (--no-exchange skips)
  inprocess     rank 0 alone drives all N GPUs through one
                fedml_amd.multidev.MultiDeviceBucket (the mode FedML's single
                server process uses; --no-inprocess skips)
  cfg4          at N >= 4: BASELINE config 4 (512 x ViT-B/16 bf16) on the
                parameter axis, the client axis (fp32 partial reduce-scatter)
                and in one process
  cfg5          at N = 8: BASELINE config 5 (64 x Llama-2-7B LoRA) FedAvg fused
                with the SGD server step (lr 1.0, momentum 0.9) through
                ShardedFedOpt (client axis + RCCL) and MultiDeviceFedOptServer
                (one process)
  (--nest overrides which config legs run: auto, none, cfg4, cfg5, cfg4,cfg5)

Robustness of the multi-GPU run: every rank meets the
others only through the rendezvous TCP store (`Coord`: barriers with a
deadline, timings gathered as JSON), so the exchange-free headline needs
neither RCCL nor gloo; the process group (120 s timeout) is used by the
nested client-axis legs alone, and RCCL creates its communicator at their
first collective.  Before that collective every rank posts "ok" or its
failure (`Leg.ready`); a leg any rank failed is abandoned by all of them, and
its object carries the error.  Rank 0 starts a nested leg only while the job
budget (--budget-s, default 480 s of the driver's 600 s) leaves that leg's
reserve, else the object says "skipped: budget".  A watchdog thread on every
rank prints whatever line rank 0 has at budget + 60 s and ends the process,
so even a collective that never returns costs the nested object, not the
line.  FEDAGG_BENCH_FAIL / FEDAGG_BENCH_HANG ("<leg>:<rank>,...") inject a
failure or a hang into a leg's handshake (tests/test_bench_legs.py, with
--probe-cpu: the same orchestration with host stand-in reductions on gloo).

Prints ONE JSON line on rank 0 (contract in the task statement); at N = 1 the
cpu_baseline leg times the reference's own CPU loop (oracle/cpu_baseline.py)
over the FULL workload (every key, every client) at the job's CPU quota and
at one thread.  `--op median` lines also carry roofline.valu: the median's
sorting networks are bound by VALU issue above ~128 clients, so the executed
VALU instructions of its kernel (profiles/median_valu.json, an SQ pass) at 4
cycles per wave64 instruction per SIMD are set against the kernel time.
"""
from __future__ import annotations

import time

T_START = time.monotonic()  # the job budget counts from here, before torch loads

import argparse  # noqa: E402
import datetime  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402
import threading  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from fedml_amd import shapes  # noqa: E402
from fedml_amd.bucket import ClientBucket  # noqa: E402
from fedml_amd import multidev  # noqa: E402
from fedml_amd.layout import RowLayout  # noqa: E402
from fedml_amd.sharded import ClientAxisAggregator  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# packed fp32 vector peak (v_pk_fma_f32: 64 FLOP/clk/SIMD x 1,024 SIMDs x 2.4 GHz), the ceiling of
# the exact-difference Krum pair kernel, whose packed subtract + packed FMA are 3 flops per client pair and
# element (the centred-Gram kernel on the bf16 matrix cores is priced against HBM instead: it reads the
# rows once; MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_TFLOPS = 157.3
SIMDS = 256 * 4  # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4
VALU_HALF_RATE_CYCLES = 4  # min/max/med3/DPP wave64 issue cost per SIMD (profiles/r03/median_rsel/valu_rate_probe*.txt)
LSA_PRIME, LSA_QBITS = 2 ** 15 - 19, 10  # the reference's example LightSecAgg config (fedml_config.yaml:58-59)
PG_TIMEOUT_S = 120.0  # process group and store timeout (RCCL's default, 10 min, outlasts the driver's limit)
WATCHDOG_GRACE_S = 60.0  # the watchdog fires this long after --budget-s

CONFIGS = {
    "cfg1": dict(model="lr_mnist", K=4, desc="FedAvg 4 clients x LogisticRegression MNIST (7,850 params) fp32"),
    "cfg2": dict(model="cnn_web", K=32, desc="FedAvg 32 clients x LeNet CNN_WEB (62,006 params) fp32"),
    "cfg3": dict(model="resnet50", K=128,
                 desc="FedAvg 128 clients x ResNet-50 state dict (25,610,152 fp32 + 53 int64) fp32"),
    "cfg4": dict(model="vit_b16", K=512, desc="FedAvg 512 clients x ViT-B/16 (86,567,656) bf16"),
    "cfg5": dict(model="llama2_7b_lora", K=64, desc="FedAvg 64 clients x Llama-2-7B LoRA r=8 q/v fp32"),
}

# seconds of job budget a nested leg must find left before rank 0 starts it
LEG_RESERVE_S = {"exchange": 45.0, "inprocess": 45.0, "cfg4/param": 60.0, "cfg4/exchange": 90.0,
                 "cfg4/inprocess": 90.0, "cfg5/sharded_fedopt": 45.0, "cfg5/inprocess_fedopt": 45.0}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="param", choices=["client", "param"],
                    help="multi-GPU partitioning (ignored at 1 GPU): param = whole keys per rank, no exchange; "
                         "client = clients per rank + RCCL reduce-scatter")
    ap.add_argument("--clients-total", type=int, default=None,
                    help="multi-GPU: clients of the round over all ranks (default: the config's K)")
    ap.add_argument("--weak", action="store_true",
                    help="multi-GPU: every rank aggregates the config's K clients of its own (weak scaling)")
    ap.add_argument("--chunks", type=int, default=8, help="client mode: reduce-scatter pipeline depth")
    ap.add_argument("--acc", default="reference", choices=["reference", "fp32"],
                    help="bf16/f16 accumulation: torch's per-op chain (bit-exact) or fp32")
    ap.add_argument("--fedopt", nargs="?", const="sgd", default=None,
                    choices=["sgd", "adam", "adamw", "adagrad", "rmsprop", "adamax", "nadam", "radam", "adadelta",
                             "asgd", "rprop"],
                    help="1 GPU: FedOpt server step fused into the reduction (config 5: SGD lr=1.0 momentum 0.9, "
                         "or the other optimizers at lr=1.0 with torch defaults)")
    ap.add_argument("--op", default="fedavg", choices=["fedavg", "median", "secagg", "lsa", "krum", "dist2", "clip",
                                                       "rlr", "mpi"],
                    help="1 GPU: the reduction measured (median = the wise_median defense kernel; secagg = "
                         "LightSecAgg's int64 sum mod p; lsa = its fused mask-cancel / de-quantize reconstruction; "
                         "krum / dist2 / clip = the distance defenses' kernels; rlr = the robust-learning-rate "
                         "defense's fused pass; mpi = the MPI simulation's fl(fl(p n_i) / N) order, "
                         "fedagg_wsum_muldiv)")
    ap.add_argument("--pair-distance", default="auto", choices=["auto", "gram", "exact"],
                    help="--op krum: the centred Gram on the bf16 matrix cores with an exact three-way split "
                         "(K <= 128) or the exact-difference VALU kernel")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = host-staged collectives, for rehearsing N ranks on one GPU (not a benchmark)")
    ap.add_argument("--clients", type=int, default=None,
                    help="1 GPU: clients per GPU instead of the config's (e.g. config 4's median over all 512 "
                         "clients: the median does not split along the client axis)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exchange", action="store_true",
                    help="multi-GPU --mode param: skip the nested client-axis (RCCL reduce-scatter) measurement")
    ap.add_argument("--cpu-reps", type=int, default=5, help="cpu_baseline: timed runs after one warm-up")
    ap.add_argument("--no-inprocess", action="store_true",
                    help="multi-GPU --mode param: skip the nested one-process measurement (MultiDeviceBucket over "
                         "the N GPUs, the mode FedML's single server process uses)")
    ap.add_argument("--nest", default="auto",
                    help="multi-GPU --mode param: the nested config legs: auto (cfg4 at N >= 4, cfg5 at N = 8), "
                         "none, or a comma list of cfg4 / cfg5")
    ap.add_argument("--budget-s", type=float, default=480.0,
                    help="multi-GPU: job seconds (from process start) within which nested legs may start; the "
                         "watchdog prints the line and ends every rank 60 s later")
    ap.add_argument("--watchdog-s", type=float, default=None, help=argparse.SUPPRESS)  # default: budget + 60 s
    ap.add_argument("--spawn-probe", action="store_true", help=argparse.SUPPRESS)  # CPU test of the self-launch
    ap.add_argument("--probe-cpu", action="store_true", help=argparse.SUPPRESS)  # CPU test of the orchestration
    return ap.parse_args(argv)


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, probe: bool = False, grace_s: float = 60.0) -> int:
    """`python bench.py --gpus N` without torch.distributed.run: start N
    worker processes of this script, one per GPU, with torchrun's environment
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), wait for them and
    return the first failing exit code (0 if all succeed).  The parent never
    touches the GPU (no HIP call before or after the spawn: the workers start
    as fresh processes, not forks), and rank 0 prints the JSON line.  Once
    rank 0 has exited cleanly (its line is out), ranks still running after
    ``grace_s`` are terminated and do not change the exit code."""
    import signal
    import subprocess

    assert not torch.cuda.is_initialized(), "the launcher must not initialise HIP"
    port = free_port()
    procs = []

    def stop_all():
        for q in procs:
            if q.poll() is None:
                q.terminate()

    def on_signal(signum, frame):  # the launcher is stopped (a time limit): take the ranks with it
        stop_all()
        raise SystemExit(128 + signum)

    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    rank0_done = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if p is procs[0] and code == 0:
                    rank0_done = time.monotonic()
                if code != 0 and rc == 0 and rank0_done is None:
                    rc = code
                    stop_all()  # a rank died: the others would wait for it until their deadlines
            if live and rank0_done is not None and time.monotonic() - rank0_done > grace_s:
                stop_all()  # the line is out; a rank that has not followed in grace_s is stuck
                for p in live:
                    p.wait()
                live = []
            time.sleep(0.05)
    finally:
        stop_all()
        for p in procs:
            p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    if probe:
        print(json.dumps({"probe": "parent", "cuda_initialized": torch.cuda.is_initialized(),
                          "exit_codes": [p.returncode for p in procs]}), flush=True)
    return rc


# ---- host-only coordination of the ranks -------------------------------------------------------------------------


class Coord:
    """Host-only coordination of the bench's ranks through the rendezvous TCP
    store: barriers with a deadline, and small JSON values gathered from
    every rank.  Nothing here touches the GPU or a collective backend, so the
    exchange-free measurements depend on neither RCCL nor gloo, and a waiting
    rank leaves no spinning kernel on its GPU.  Every name is used once per
    run (keys are never reused).  The first deadline that passes marks the
    coordination broken: later nested legs are skipped, not waited for."""

    def __init__(self, world: int, rank: int, store=None, timeout_s: float = PG_TIMEOUT_S):
        self.world, self.rank, self.store, self.timeout_s = world, rank, store, timeout_s
        self.broken = None
        self._used = set()

    def _key(self, name: str) -> str:
        if name in self._used:
            raise ValueError(f"coordination name {name!r} used twice")
        self._used.add(name)
        return "bench/" + name

    def _deadline(self, timeout_s):
        return time.monotonic() + (self.timeout_s if timeout_s is None else timeout_s)

    def _timeout(self, what: str) -> TimeoutError:
        self.broken = self.broken or what
        return TimeoutError(what)

    def barrier(self, name: str, timeout_s=None) -> None:
        if self.world == 1:
            return
        key = self._key(name)
        self.store.add(key, 1)
        deadline = self._deadline(timeout_s)
        while True:
            n = self.store.add(key, 0)
            if n >= self.world:
                return
            if time.monotonic() > deadline:
                raise self._timeout(f"barrier {name!r}: {n} of {self.world} ranks arrived in time")
            time.sleep(0.005)

    def post(self, name: str, value) -> None:
        """This rank's value under ``name`` (collect() reads every rank's)."""
        if self.world > 1:
            self.store.set(f"bench/{name}/{self.rank}", json.dumps(value))

    def collect(self, name: str, timeout_s=None, abort_key=None) -> list:
        """Every rank's posted value under ``name``, in rank order.  abort_key:
        a store key whose appearance ends the wait with LegAborted (a rank
        that failed mid-leg posts it)."""
        if self.world == 1:
            raise ValueError("collect() needs ranks")
        self._key(name)
        keys = [f"bench/{name}/{r}" for r in range(self.world)]
        deadline = self._deadline(timeout_s)
        while not self.store.check(keys):
            if abort_key is not None and self.store.check([abort_key]):
                raise LegAborted(self.store.get(abort_key).decode())
            if time.monotonic() > deadline:
                have = [r for r, k in enumerate(keys) if self.store.check([k])]
                raise self._timeout(f"{name!r}: only ranks {have} of {self.world} posted in time")
            time.sleep(0.005)
        return [json.loads(self.store.get(k)) for k in keys]

    def allgather(self, name: str, value, timeout_s=None, abort_key=None) -> list:
        if self.world == 1:
            return [value]
        self.post(name, value)
        return self.collect(name, timeout_s, abort_key)

    def from_rank0(self, name: str, value, timeout_s=None):
        """Rank 0's value, on every rank (rank 0 decides, the others follow)."""
        if self.world == 1:
            return value
        key = self._key(name)
        if self.rank == 0:
            self.store.set(key, json.dumps(value))
            return value
        deadline = self._deadline(timeout_s)
        while not self.store.check([key]):
            if time.monotonic() > deadline:
                raise self._timeout(f"{name!r}: rank 0 did not decide in time")
            time.sleep(0.005)
        return json.loads(self.store.get(key))


SOLO = Coord(1, 0)


def host_barrier(tag: str, world: int, timeout_s: float = PG_TIMEOUT_S) -> None:
    """A host-only barrier on the default process group's store, with a
    deadline (TimeoutError)."""
    store = dist.distributed_c10d._get_default_store()
    Coord(world, dist.get_rank(), store).barrier(tag, timeout_s)


class LegAborted(RuntimeError):
    """A leg abandoned by this rank because another rank failed in it."""


def _injected(kind: str, name: str, rank: int) -> bool:
    """FEDAGG_BENCH_<kind> = "<leg>:<rank>,...": the test hooks."""
    for item in os.environ.get(f"FEDAGG_BENCH_{kind}", "").split(","):
        leg, _, r = item.strip().rpartition(":")
        if leg == name and r.isdigit() and int(r) == rank:
            return True
    return False


class Leg:
    """One measurement of the run as the ranks see it: coordination names
    under the leg's name, the readiness handshake before its first
    collective, and the abort key a failing rank posts."""

    def __init__(self, coord: Coord, name: str):
        self.coord, self.name = coord, name
        self.abort_key = f"bench/{name}/abort"
        self._posted = False

    @property
    def rank(self) -> int:
        return self.coord.rank

    @property
    def world(self) -> int:
        return self.coord.world

    def barrier(self, tag: str, timeout_s=None) -> None:
        self.coord.barrier(f"{self.name}/{tag}", timeout_s)

    def allgather(self, tag: str, value, timeout_s=None) -> list:
        return self.coord.allgather(f"{self.name}/{tag}", value, timeout_s, self.abort_key)

    def ready(self) -> None:
        """Handshake before the leg's first collective: every rank posts "ok"
        once its rows are allocated and filled, or its failure (``fail``).
        If any rank failed, every rank abandons the leg here, before anyone
        enters the collective that would wait for the failed rank."""
        if _injected("FAIL", self.name, self.rank):
            raise RuntimeError(f"injected failure (FEDAGG_BENCH_FAIL) in {self.name} on rank {self.rank}")
        if self.world > 1:
            self._posted = True
            states = self.coord.allgather(f"{self.name}/ready", "ok")
            bad = [f"rank {r}: {s}" for r, s in enumerate(states) if s != "ok"]
            if bad:
                raise LegAborted("; ".join(bad) + " -- every rank skipped the leg's collective")
        if _injected("HANG", self.name, self.rank):  # a rank lost inside the collective phase
            while True:
                time.sleep(3600)

    def fail(self, msg: str) -> None:
        """This rank failed in the leg: answer the handshake (if not yet) and
        post the abort key, so no rank waits for it."""
        if self.world == 1:
            return
        if not self._posted:
            self._posted = True
            self.coord.post(f"{self.name}/ready", f"failed: {msg}")
        self.coord.store.set(self.abort_key, f"rank {self.rank}: {msg}")


class Budget:
    def __init__(self, total_s: float):
        self.total_s = total_s

    def left(self) -> float:
        return self.total_s - (time.monotonic() - T_START)


class Report:
    """The line being built (rank 0), printed exactly once: normally at the
    end of main, or by the watchdog with what is there."""

    def __init__(self):
        self.line = None
        self.leg = None
        self._lock = threading.Lock()
        self._printed = False

    def emit(self, extra=None) -> bool:
        with self._lock:
            if self._printed or self.line is None:
                return False
            if extra:
                self.line.update(extra)
            print(json.dumps(self.line), flush=True)
            self._printed = True
            return True


REPORT = Report()


def start_watchdog(rank: int, budget: Budget, at_s=None) -> threading.Timer:
    """After budget + grace, rank 0 prints the line as it stands (the running
    leg marked) and every rank ends: a collective that never returns must
    not cost the line or outlast the driver's limit."""
    def fire():
        running = REPORT.leg
        if rank == 0:
            REPORT.emit({"watchdog": f"fired at {time.monotonic() - T_START:.0f} s; still running: {running}"})
        sys.stdout.flush()
        sys.stderr.write(f"bench rank {rank}: watchdog fired during {running}\n")
        sys.stderr.flush()
        os._exit(0)

    at = budget.total_s + WATCHDOG_GRACE_S if at_s is None else at_s  # seconds from the job's start
    t = threading.Timer(max(1.0, at - (time.monotonic() - T_START)), fire)
    t.daemon = True
    t.start()
    return t


def run_leg(coord: Coord, budget: Budget, name: str, fn, reserve_s: float, rank0_only: bool = False,
            cleanup=None) -> dict:
    """One nested leg on every rank: rank 0 decides from the budget whether it
    starts; ``fn(leg)`` runs (on rank 0 alone if rank0_only, the others
    waiting at the end barrier); an exception becomes the leg's "error" and
    is posted so no rank waits for this one.  Every rank leaves together."""
    REPORT.leg = name
    if coord.broken:
        return {"skipped": f"coordination lost earlier ({coord.broken})"}
    left = budget.left()
    go = "run" if left >= reserve_s else f"budget: {left:.0f} s of the job budget left, the leg reserves {reserve_s:.0f} s"
    try:
        go = coord.from_rank0(f"{name}/go", go)
    except TimeoutError as e:
        return {"skipped": str(e)}
    if go != "run":
        return {"skipped": go}
    leg = Leg(coord if not rank0_only else SOLO, name)
    out = {}
    try:
        if not rank0_only or coord.rank == 0:
            out = fn(leg)
    except LegAborted as e:
        out = {"error": f"rank {coord.rank} abandoned the leg: {e}"}
    except Exception as e:  # noqa: BLE001 -- the headline stands; the leg reports what it hit
        msg = f"{type(e).__name__}: {e}"
        if not rank0_only:
            leg.fail(msg)
        out = {"error": f"rank {coord.rank}: {msg}"}
    finally:
        if cleanup is not None:
            cleanup()
    try:
        coord.barrier(f"{name}/end", max(PG_TIMEOUT_S, budget.left() + WATCHDOG_GRACE_S) if rank0_only else None)
    except TimeoutError as e:
        out.setdefault("error", str(e))
    REPORT.leg = None
    return out


# ---- workload ------------------------------------------------------------------------------------------------------


def plan_clients(config: str, world: int, rank: int, mode: str, clients_total=None, weak: bool = False,
                 clients=None):
    """(K_total, K_loc, first): the round's clients over all ranks, this
    rank's count and the index of its first client.  mode is "single" at one
    GPU, else "param" (every rank holds its keys of ALL clients) or "client"
    (clients dealt to ranks, the first K_total % world ranks one more)."""
    K = CONFIGS[config]["K"]
    if clients is not None:
        if world > 1 or clients < 1:
            raise SystemExit("--clients is a 1-GPU override (>= 1)")
        K = clients
    weak = weak and world > 1
    if world > 1 and not weak:
        K_total = clients_total if clients_total is not None else K
        if K_total < 1:
            raise SystemExit("--clients-total must be >= 1")
    else:
        K_total = K * world
    if mode == "client" and not weak:
        base_k, extra = divmod(K_total, world)
        K_loc = base_k + (1 if rank < extra else 0)
        first = rank * base_k + min(rank, extra)
    elif mode == "client" or weak:
        K_loc, first = K, rank * K
    else:
        K_loc, first = K_total, 0
    if K_loc < 1:
        raise SystemExit(f"rank {rank} would hold no clients: --clients-total {K_total} < --gpus {world}")
    return K_total, K_loc, first


def fill_rows(rows: torch.Tensor, length: int, seed: int, round_idx: int = 0) -> None:
    """Synthetic updates in HBM: base ~ N(0, 0.05²), client_i = base + 0.01·ε_i
    (SURVEY.md §8(d)); int64 rows get round_idx + i."""
    K = rows.shape[0]
    if rows.dtype == torch.int64:
        for i in range(K):
            rows[i].fill_(round_idx + i)
        return
    g = torch.Generator(device=rows.device).manual_seed(seed)
    base = torch.randn(length, generator=g, device=rows.device) * 0.05
    eps = torch.empty(length, device=rows.device)
    for i in range(K):
        eps.normal_(0.0, 1.0, generator=g)
        rows[i, :length].copy_(base + 0.01 * eps)
        rows[i, length:].zero_()
    del base, eps


def fill_bucket(bucket, seed_base: int) -> None:
    with torch.cuda.device(bucket.device):
        for gi, (dt, g) in enumerate(bucket.groups.items()):
            fill_rows(g.rows, g.length, seed=seed_base + gi, round_idx=3)


def model_entries(config: str):
    return shapes.MODELS[CONFIGS[config]["model"]]()


def elements_per_client(entries) -> int:
    return sum(sum(g.numels) for g in RowLayout(entries).groups.values())


CPU_SAMPLE_BYTES = 13_400_000_000  # cpu_baseline: client bytes copied to the host (config 3 = 13.2 GB, all of it)


def host_round(bucket, clients=None) -> list:
    """The bench's round as the reference's CPU server holds it: K pageable
    per-key host tensors per client (contiguous slices of one host copy of
    each client's row; integer keys as int64 tensors), copied from HBM.
    clients: the first this many slots (default all)."""
    from collections import OrderedDict

    raw = []
    for i in range(bucket.capacity if clients is None else clients):
        d = OrderedDict()
        rows = {dt: g.rows[i, :g.length].cpu() for dt, g in bucket.groups.items()}
        for key, shape, dt in bucket.entries:
            g, j = bucket.where[key]
            t = rows[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].view(shape)
            d[key] = t.to(dt) if key in bucket.int_keys else t
        raw.append((bucket.sample_nums[i] if bucket.sample_nums[i] is not None else 1, d))
    return raw


def cpu_baseline(bucket, ns, reps: int) -> dict:
    """The reference's own CPU loop (agg_operator.py:35-44 in torch eager,
    oracle/cpu_baseline.py) on every key of the state dict and the same values
    as the HBM rows: all K clients while they fit CPU_SAMPLE_BYTES (config 3:
    the FULL workload), else the first K' clients that do (config 4's 512 x
    173 MB: a bounded sample; the unit is a rate, client-params/s).  Median of
    `reps` runs after one warm-up, at every CPU this job may use and at one
    thread."""
    from oracle import cpu_baseline as cb

    row_bytes = sum(g.length * g.rows.element_size() for g in bucket.groups.values())
    k_all = bucket.capacity
    k_s = max(1, min(k_all, CPU_SAMPLE_BYTES // max(1, row_bytes)))
    raw = host_round(bucket, k_s)
    raw = [(n, d) for n, (_, d) in zip(ns, raw)]
    cpus = cb.host_cpus()
    full = cb.time_fedavg(raw, reps=reps, threads=cpus["usable"])
    one = cb.time_fedavg(raw, reps=reps, threads=1)
    K = len(raw)
    n_elems = bucket.num_elements()
    del raw
    return {"value": K * n_elems / full["median_s"], "unit": "client-params/s", "cores": full["threads"],
            "kind": "port",
            "sample": ("full workload" if K == k_all else f"bounded sample: the first {K} of {k_all} clients") +
                      f": all {len(bucket.entries)} state-dict keys x {K} clients "
                      f"({n_elems:,} elements/client), torch-eager restatement of agg_operator.py:35-44, "
                      f"median of {reps} after 1 warm-up: {full['median_s'] * 1e3:.1f} ms/aggregation at "
                      f"{full['threads']} threads, {one['median_s'] * 1e3:.1f} ms at 1 thread",
            "threads": full["threads"],
            "cores_basis": "threads used = the CPUs this job may use (the box's cgroup quota), not the host's "
                           "nproc; see host",
            "ms_per_aggregation": round(full["median_s"] * 1e3, 2),
            "single_thread": {"value": K * n_elems / one["median_s"], "threads": 1,
                              "ms_per_aggregation": round(one["median_s"] * 1e3, 2)},
            "host": {"cpu_model": cpus["model"], "nproc": cpus["nproc"], "affinity_cpus": cpus["affinity"],
                     "cgroup_quota_cpus": cpus["cgroup_quota_cpus"]}}


def median_kernel_name(K: int, dt) -> str:
    """The kernel fedagg_median dispatches for K clients of aligned rows
    (median_dispatch in csrc/median.hip)."""
    name = str(dt).replace("torch.", "")
    packed = dt in (torch.bfloat16, torch.float16)
    if packed and 96 < K <= 128:  # bit-plane select, one lane per column pair
        return f"median_pk16_lanes_kernel<1, 128, planes> ({name})"
    if K <= 128:
        kmax = next(m for m in ((32, 64, 96, 128) if packed else (8, 16, 24, 32, 48, 64, 96, 128)) if K <= m)
        return f"median_{'pk16_' if packed else ''}kernel<{kmax}> ({name})"
    if K > 4096 or (not packed and 2048 < K <= 2560):
        return f"median_radix_stream_kernel ({name})"
    if packed and K <= 1024:  # streamed bit-plane select, one column per lane (+ the register form for the tail)
        p, w = (2, 4) if K <= 256 else (4, 4) if K <= 512 else (8, 8)
        return f"median_pk16_colstream_kernel<{p}, 64, {w}> ({name})"
    p, r = (4, 64) if K <= 256 else (4, 128) if K <= 512 else (8, 128) if K <= 1024 else \
        (16, 128) if K <= 2048 else (32, 128)
    return f"median_{'pk16_' if packed else ''}lanes_kernel<{p}, {r}> ({name})"


def table_key(config: str, mode: str, world: int, variant: str, clients: int) -> str:
    """Key of a measurement table entry: config, partitioning, variant and the
    clients per GPU it was measured at, e.g. "cfg4:single@K512",
    "cfg3:single:median@K128"."""
    return f"{config}:{mode if world > 1 else 'single'}" + (f":{variant}" if variant else "") + f"@K{clients}"


def load_traffic(config: str, mode: str, world: int, variant: str = "", clients: int = 128):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None.
    variant: "" for FedAvg, else the fused server step or the robust op."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = table_key(config, mode, world, variant, clients)
    try:
        return json.load(open(path)).get(key, {}).get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_median_valu(config: str, mode: str, world: int, variant: str, clients: int):
    """Executed VALU instructions per wave and waves per launch of the median
    kernel at this shape, from the committed SQ pass (profiles/median_valu.json,
    tools/median_valu.py), or None."""
    path = os.path.join(ROOT, "profiles", "median_valu.json")
    key = table_key(config, mode, world, variant, clients)
    try:
        return json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None


# ---- timing ---------------------------------------------------------------------------------------------------------


class HostEvent:
    """torch.cuda.Event's timing interface on the host clock (--probe-cpu)."""

    def __init__(self, enable_timing=True):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, end) -> float:
        return (end.t - self.t) * 1e3


def _cuda_event():
    return torch.cuda.Event(enable_timing=True)


def run_timed(step, n_launch: int, steps: int, warmup: int, leg: Leg, per_chunk: bool, timed_comm: bool,
              sync=None, event=None):
    """W untimed steps, then K timed steps between a host barrier (the
    rendezvous store) + synchronize on both sides.  Returns this rank's
    (elapsed s; kernel ms per step from the events on the launch stream;
    comm-stream ms per step or None); ``over_ranks`` combines them."""
    sync = sync or torch.cuda.synchronize
    event = event or _cuda_event

    def new_events(n):
        return [[event(), event()] for _ in range(n)]

    for _ in range(warmup):
        step()
    evs = [new_events(n_launch) for _ in range(steps)]
    cevs = [new_events(n_launch) for _ in range(steps)] if timed_comm else [None] * steps
    sync()
    leg.barrier("start")
    t0 = time.perf_counter()
    for s in range(steps):
        # the client-axis steps take one (start, end) pair per chunk; the rest one pair
        step(evs[s] if per_chunk else evs[s][0], cevs[s])
    sync()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(e0.elapsed_time(e1) for ev in evs for e0, e1 in ev) / steps  # per step
    comm_ms = sum(e0.elapsed_time(e1) for ev in cevs for e0, e1 in ev) / steps if timed_comm else None
    return elapsed, kern_ms, comm_ms


def over_ranks(leg: Leg, elapsed: float, achieved: float, hbm: float, comm_ms):
    """Through the store: the MAX elapsed over ranks, the slowest rank's kernel
    rate, the sum of the ranks' HBM rates and the mean comm-stream time."""
    rows = leg.allgather("timing", [elapsed, achieved, hbm, comm_ms])
    comm = [r[3] for r in rows if r[3] is not None]
    return (max(r[0] for r in rows), min(r[1] for r in rows), sum(r[2] for r in rows),
            sum(comm) / len(comm) if comm else None)


# ---- nested legs (GPU) ---------------------------------------------------------------------------------------------


def leg_steps(a):
    """Steps of a nested collective leg: the run's, or 3 + 1 on gloo (a
    host-staged rehearsal whose reduce-scatter costs ~0.1-1 s per step)."""
    return (min(a.steps, 3), min(a.warmup, 1)) if a.backend == "gloo" else (a.steps, a.warmup)


def measure_param(a, config: str, leg: Leg, dev) -> dict:
    """A config's parameter axis over the ranks: this rank's whole keys
    (multidev.shard_plan) of all K clients, reduced in the reference order;
    no collective, bit-exact with one GPU."""
    from fedml_amd.synth import sample_nums

    world, rank = leg.world, leg.rank
    entries = model_entries(config)
    K = CONFIGS[config]["K"]
    plan = multidev.shard_plan(entries, world)
    if len(plan) < world:
        return {"skipped": f"{config} has data in {len(plan)} keys: too few for {world} ranks"}
    bucket = ClientBucket(plan[rank], K, dev, low_precision_acc=a.acc)
    fill_bucket(bucket, 1000 * rank)
    ns = sample_nums(K, seed=1)
    w = bucket.weights(ns)
    outs = bucket.new_outputs()
    dom = bucket.dominant_dtype()

    def step(ev=None, cev=None):
        bucket.reduce_into(outs, w, events={dom: ev} if ev is not None else None)

    torch.cuda.synchronize()
    leg.ready()
    elapsed, kern_ms, _ = run_timed(step, 1, a.steps, a.warmup, leg, False, False)
    gd = bucket.groups[dom]
    dom_bytes = K * gd.length * gd.rows.element_size() + gd.length * torch.empty((), dtype=gd.out_dtype).element_size()
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9
    hbm = bucket.algorithmic_bytes() / (elapsed / a.steps) / 1e9
    elapsed, achieved, hbm, _ = over_ranks(leg, elapsed, achieved, hbm, None)
    n_elems = elements_per_client(entries)
    return {"mode": "param", "workload": CONFIGS[config]["desc"], "world_size": world, "clients_total": K,
            "value": K * n_elems / (elapsed / a.steps), "unit": "client-params/s",
            "ms_per_step": elapsed / a.steps * 1e3, "kernel_gbps_slowest_rank": round(achieved, 1),
            "frac_slowest_rank": round(achieved / HBM_PEAK_GBPS, 4), "aggregate_gbps": round(hbm, 1),
            "aggregate_frac_of_n_peaks": round(hbm / (world * HBM_PEAK_GBPS), 4),
            "parity": "bit-exact with one GPU (whole keys per rank, reference client order)"}


def measure_client_axis(a, config: str, leg: Leg, dev) -> dict:
    """north_star's client-axis mode on a config's round (its K clients and
    sample counts): this rank's K/world clients' whole updates, the fp32
    partial and the chunked RCCL reduce-scatter over xGMI; 16-bit models
    round once after the exchange."""
    from fedml_amd.synth import sample_nums

    world, rank = leg.world, leg.rank
    K_total = CONFIGS[config]["K"] if config != a.config or a.clients_total is None else a.clients_total
    entries = model_entries(config)
    if K_total < world:
        return {"mode": "client", "skipped": f"{K_total} clients cannot cover {world} ranks on the client axis"}
    _, K_c, first_c = plan_clients(config, world, rank, "client", K_total)
    ns_all = sample_nums(K_total, seed=1)
    total_n = sum(ns_all)
    w = [n / total_n for n in ns_all[first_c:first_c + K_c]]
    bucket = ClientBucket(entries, K_c, dev, low_precision_acc=a.acc)
    fill_bucket(bucket, 1000 * rank)
    torch.cuda.synchronize()
    dom_dt = bucket.dominant_dtype()
    step, n_launch, dom_bytes, xgmi_bytes = client_axis_step(bucket, dom_dt, w, a.chunks, world)
    backend = dist.get_backend()
    timed_comm = backend == "nccl"
    steps, warmup = leg_steps(a)
    leg.ready()  # every rank's rows are filled: only now does anyone enter the collective
    elapsed, kern_ms, comm_ms = run_timed(step, n_launch, steps, warmup, leg, True, timed_comm)
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9
    hbm_all = dom_bytes / (elapsed / steps) / 1e9
    elapsed, achieved, hbm_all, comm_ms = over_ranks(leg, elapsed, achieved, hbm_all, comm_ms)
    ms = elapsed / steps * 1e3
    n_elems = elements_per_client(entries)
    rehearsal = backend != "nccl"
    return {"mode": "client", "workload": CONFIGS[config]["desc"], "backend": backend, "world_size": world,
            "collective": "reduce_scatter_tensor (RCCL over xGMI)" if not rehearsal else
            "reduce_scatter_tensor (gloo, host-staged: a rehearsal, not a measurement)",
            "clients_total": K_total, "clients_per_gpu": K_c, "chunks": n_launch, "steps": steps,
            "value": K_total * n_elems / (elapsed / steps), "unit": "client-params/s",
            "ms_per_step": ms, "kernel_ms_per_step": round(kern_ms, 4),
            "kernel_gbps_slowest_rank": round(achieved, 1), "frac_slowest_rank": round(achieved / HBM_PEAK_GBPS, 4),
            "aggregate_gbps": round(hbm_all, 1), "xgmi_bytes_per_rank_per_step": xgmi_bytes,
            "comm_ms_per_step": round(comm_ms, 4) if comm_ms is not None else None,
            "parity": "fp32 partials summed across GPUs: |d| <= 2(K + log2 G + 1) 2^-24 sum|w_i p_i| vs one GPU "
                      "(ClientAxisAggregator.tolerance; tests/test_sharded_gloo.py)",
            "note": "comm_ms: mean over ranks of the chunks' reduce-scatter time on the comm stream (overlapping "
                    "the next chunk's reduction)"}


def client_axis_step(bucket, dom_dt, w_local, chunks: int, world: int):
    """The client-axis step over this rank's bucket: per dtype group the fp32
    partial of its clients (global weights) and the chunked reduce-scatter,
    16-bit models rounded once after the exchange.  Returns (step, launches
    per step of the dominant group, its algorithmic bytes, xGMI bytes per rank)."""
    aggs = {dt: ClientAxisAggregator(g.rows, g.length, chunks=chunks if dt == dom_dt else 1)
            for dt, g in bucket.groups.items()}

    def step(ev=None, cev=None):
        for dt, agg in aggs.items():
            agg.aggregate(w_local, events=ev if dt == dom_dt else None,
                          comm_events=cev if dt == dom_dt else None)
            if dt in (torch.bfloat16, torch.float16):
                agg.shard_in_model_dtype()  # the one rounding of a 16-bit model, after the exchange

    gd = bucket.groups[dom_dt]
    dom_bytes = gd.rows.shape[0] * gd.length * gd.rows.element_size() + gd.length * 4  # rows in, fp32 partial out
    xgmi_bytes = (world - 1) * aggs[dom_dt].piece * len(aggs[dom_dt].bounds) * 4
    return step, len(aggs[dom_dt].bounds), dom_bytes, xgmi_bytes


def _inprocess_devices(world: int):
    n_dev = torch.cuda.device_count()
    return [torch.device("cuda", i % n_dev) for i in range(world)]


def _sync_devices(devices) -> None:
    for i in sorted({d.index for d in devices}):
        torch.cuda.synchronize(i)


def measure_inprocess(a, config: str, world: int) -> dict:
    """The multi-GPU mode FedML's server can use: ONE process (the server is
    one process, python/fedml/__init__.py:330-348) driving `world` GPUs
    through fedml_amd.multidev.MultiDeviceBucket: whole keys per device, every
    device reducing its keys of all K clients in the reference order (no
    exchange, bit-exact with one GPU; cross_silo/server/fedml_aggregator.py:
    58-67 feeds it).  Device-resident rows, the same clients and weights as
    the parameter axis; runs on rank 0 while the other ranks wait at a host
    barrier with their rows freed."""
    from fedml_amd.synth import sample_nums

    entries = model_entries(config)
    K_total = CONFIGS[config]["K"] if config != a.config or a.clients_total is None else a.clients_total
    mb = multidev.MultiDeviceBucket(entries, K_total, _inprocess_devices(world), low_precision_acc=a.acc)
    for s, b in enumerate(mb.shards):
        fill_bucket(b, 5000 + 100 * s)
    ns = sample_nums(K_total, seed=1)
    w = mb.weights(ns)
    outs = [b.new_outputs() for b in mb.shards]
    doms = [b.dominant_dtype() for b in mb.shards]

    def step(evs=None):
        # every device's launch in one native call (MultiDeviceBucket.reduce_into_all), or shard by shard
        if not mb.reduce_into_all(outs, w, events=evs):
            for s, b in enumerate(mb.shards):
                b.reduce_into(outs[s], w, events={doms[s]: evs[s]} if evs is not None else None)

    for _ in range(a.warmup):
        step()
    evs = []
    for _ in range(a.steps):
        per = []
        for b in mb.shards:
            with torch.cuda.device(b.device):
                per.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        evs.append(per)
    _sync_devices(mb.devices)
    t0 = time.perf_counter()
    for s in range(a.steps):
        step(evs[s])
    _sync_devices(mb.devices)
    elapsed = time.perf_counter() - t0
    per_dev = []
    total_bytes = 0
    for s, b in enumerate(mb.shards):
        g = b.groups[doms[s]]
        dom_bytes = K_total * g.length * g.rows.element_size() + \
            g.length * torch.empty((), dtype=g.out_dtype).element_size()
        kern_ms = sum(ev[s][0].elapsed_time(ev[s][1]) for ev in evs) / a.steps
        gbps = dom_bytes / (kern_ms / 1e3) / 1e9
        total_bytes += b.algorithmic_bytes()
        per_dev.append({"device": str(b.device), "keys": len(b.entries), "alg_bytes_per_step": dom_bytes,
                        "kernel_ms_per_step": round(kern_ms, 4), "gbps": round(gbps, 1),
                        "frac": round(gbps / HBM_PEAK_GBPS, 4)})
    ms = elapsed / a.steps * 1e3
    used = {d.index for d in mb.devices}
    shared = len(used) < len(mb.shards)
    n_elems = elements_per_client(entries)
    return {"mode": "one process, G GPUs (fedml_amd.multidev.MultiDeviceBucket)", "workload": CONFIGS[config]["desc"],
            "devices": len(mb.shards), "distinct_gpus": len(used), "clients_total": K_total,
            "value": K_total * n_elems / (elapsed / a.steps), "unit": "client-params/s", "ms_per_step": ms,
            "slowest_device_kernel_ms": max(d["kernel_ms_per_step"] for d in per_dev),
            "per_device": per_dev, "aggregate_gbps": round(total_bytes / (elapsed / a.steps) / 1e9, 1),
            "aggregate_frac_of_n_peaks": round(total_bytes / (elapsed / a.steps) / 1e9 / (len(used) * HBM_PEAK_GBPS),
                                               4),
            "shard_balance": round(max(mb.shard_bytes()) / (sum(mb.shard_bytes()) / len(mb.shards)), 4),
            "parity": "bit-exact with one GPU (whole keys per device, reference client order; "
                      "tests/test_gpu_multidev.py)",
            "note": ("shards share one GPU here: a rehearsal of the launch pattern, not a multi-GPU rate"
                     if shared else "device-resident rows; reduce_to_host (D2H) excluded, as in the headline")}


CFG5_STEP = ("sgd", 1.0, 0.9)  # config 5's server step in the nested legs: SGD lr 1.0 momentum 0.9


def measure_sharded_fedopt(a, config: str, leg: Leg, dev) -> dict:
    """Config 5 over the ranks' client axis: ShardedFedOpt (fp32 partial,
    chunked RCCL reduce-scatter, then the fused SGD + momentum step on each
    rank's 1/G shard with sharded optimizer state)."""
    from fedml_amd.sharded import ShardedFedOpt, buffer_ranges
    from fedml_amd.synth import sample_nums

    world, rank = leg.world, leg.rank
    entries = model_entries(config)
    K_total = CONFIGS[config]["K"]
    if K_total < world:
        return {"skipped": f"{K_total} clients cannot cover {world} ranks on the client axis"}
    _, K_c, first_c = plan_clients(config, world, rank, "client", K_total)
    ns_all = sample_nums(K_total, seed=1)
    total_n = sum(ns_all)
    w = [n / total_n for n in ns_all[first_c:first_c + K_c]]
    bucket = ClientBucket(entries, K_c, dev)
    if set(bucket.groups) != {torch.float32}:
        return {"skipped": f"{config}: the sharded FedOpt leg takes an fp32 model"}
    fill_bucket(bucket, 1000 * rank)
    gd = bucket.groups[torch.float32]
    init = torch.zeros(gd.length, dtype=torch.float32, device=dev)
    opt_name, lr, mom = CFG5_STEP
    opt = ShardedFedOpt(gd.rows, gd.length, init, opt_name, lr, mom, chunks=a.chunks,
                        buffers=buffer_ranges(bucket, shapes.param_names(entries)))
    torch.cuda.synchronize()
    steps, warmup = leg_steps(a)
    leg.ready()
    opt.aggregate(w)  # the first step (no momentum read) before timing

    def step(ev=None, cev=None):
        opt.aggregate(w, events=ev, comm_events=cev)

    timed_comm = dist.get_backend() == "nccl"
    n_launch = len(opt.agg.bounds)
    elapsed, kern_ms, comm_ms = run_timed(step, n_launch, steps, warmup, leg, True, timed_comm)
    dom_bytes = K_c * gd.length * 4 + gd.length * 4  # rows in, fp32 partial out (the step itself is 1/G of a pass)
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9
    hbm = dom_bytes / (elapsed / steps) / 1e9
    elapsed, achieved, hbm, comm_ms = over_ranks(leg, elapsed, achieved, hbm, comm_ms)
    xgmi = (world - 1) * opt.agg.piece * n_launch * 4
    n_elems = elements_per_client(entries)
    return {"mode": "client axis + sharded server step (fedml_amd.sharded.ShardedFedOpt)",
            "workload": CONFIGS[config]["desc"], "server_step": "SGD lr=1.0 momentum=0.9, each rank's 1/G shard",
            "backend": dist.get_backend(), "world_size": world, "clients_total": K_total, "clients_per_gpu": K_c,
            "steps": steps, "value": K_total * n_elems / (elapsed / steps), "unit": "client-params/s",
            "ms_per_step": elapsed / steps * 1e3, "kernel_ms_per_step": round(kern_ms, 4),
            "kernel_gbps_slowest_rank": round(achieved, 1), "frac_slowest_rank": round(achieved / HBM_PEAK_GBPS, 4),
            "xgmi_bytes_per_rank_per_step": xgmi,
            "comm_ms_per_step": round(comm_ms, 4) if comm_ms is not None else None,
            "parity": "the client-axis tolerance for the average, then the one-GPU fused step "
                      "(tests/test_gpu_multirank.py, tests/test_sharded_gloo.py)"}


def measure_inprocess_fedopt(a, config: str, world: int) -> dict:
    """Config 5 in ONE server process over `world` GPUs:
    MultiDeviceFedOptServer (whole keys per device, each device's FedAvg
    fused with the SGD + momentum step, bit-exact with one GPU)."""
    from collections import OrderedDict

    from fedml_amd.fedopt import MultiDeviceFedOptServer
    from fedml_amd.synth import sample_nums

    entries = model_entries(config)
    K = CONFIGS[config]["K"]
    devices = _inprocess_devices(world)
    init = OrderedDict((k, torch.zeros(s, dtype=d)) for k, s, d in entries)
    opt_name, lr, mom = CFG5_STEP
    server = MultiDeviceFedOptServer(init, shapes.param_names(entries), K, opt_name, lr, mom, devices)
    for s, srv in enumerate(server.servers):
        fill_bucket(srv.bucket, 7000 + 100 * s)
    for i, n in enumerate(sample_nums(K, seed=1)):
        server.sample_num_dict[i] = n
    server.aggregate()  # the first step (no momentum read) before timing
    for _ in range(a.warmup):
        server.aggregate()
    evs = []
    for _ in range(a.steps):
        per = []
        for srv in server.servers:
            with torch.cuda.device(srv.device):
                per.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        evs.append(per)
    _sync_devices(server.devices)
    t0 = time.perf_counter()
    for s in range(a.steps):
        server.aggregate(device_events=evs[s])
    _sync_devices(server.devices)
    elapsed = time.perf_counter() - t0
    per_dev = []
    for s, srv in enumerate(server.servers):
        kern_ms = sum(ev[s][0].elapsed_time(ev[s][1]) for ev in evs) / a.steps
        b = srv.algorithmic_bytes()
        per_dev.append({"device": str(srv.device), "keys": len(srv.bucket.entries), "alg_bytes_per_step": b,
                        "kernel_ms_per_step": round(kern_ms, 4), "gbps": round(b / (kern_ms / 1e3) / 1e9, 1),
                        "frac": round(b / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)})
    total = server.algorithmic_bytes()
    used = {d.index for d in server.devices}
    n_elems = elements_per_client(entries)
    return {"mode": "one process, G GPUs (fedml_amd.fedopt.MultiDeviceFedOptServer)",
            "workload": CONFIGS[config]["desc"], "server_step": "SGD lr=1.0 momentum=0.9 fused into the reduction",
            "devices": len(server.servers), "distinct_gpus": len(used), "clients_total": K,
            "value": K * n_elems / (elapsed / a.steps), "unit": "client-params/s",
            "ms_per_step": elapsed / a.steps * 1e3, "per_device": per_dev,
            "aggregate_gbps": round(total / (elapsed / a.steps) / 1e9, 1),
            "aggregate_frac_of_n_peaks": round(total / (elapsed / a.steps) / 1e9 / (len(used) * HBM_PEAK_GBPS), 4),
            "parity": "bit-exact with one GPU (tests/test_gpu_multidev_fedopt.py)",
            "note": ("shards share one GPU here: a rehearsal of the launch pattern, not a multi-GPU rate"
                     if len(used) < len(server.servers) else "device-resident rows and state")}


def _free_device_memory() -> None:
    if torch.cuda.is_initialized():
        for i in range(torch.cuda.device_count()):
            torch.cuda.synchronize(i)
        torch.cuda.empty_cache()


# ---- nested legs (--probe-cpu: host stand-ins, same orchestration) ---------------------------------------------------


PROBE_K, PROBE_N = 8, 4096


def _probe_rows(K: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn(K, PROBE_N, generator=g)


def _probe_step(fn):
    """A stand-in step recording its events on the host clock."""
    def step(ev=None, cev=None):
        if ev is not None:
            ev[0].record()
        fn()
        if ev is not None:
            ev[1].record()
    return step


def _probe_reducer(rows, weights, out):
    acc = torch.zeros(rows.shape[1], dtype=torch.float32)
    for i, wi in enumerate(weights):
        acc += rows[i].float() * wi
    out.copy_(acc)


def probe_param(a, config: str, leg: Leg, dev) -> dict:
    from fedml_amd.sharded import ParamAxisAggregator

    rows = _probe_rows(PROBE_K, 10 + leg.rank)
    agg = ParamAxisAggregator(rows, PROBE_N, reducer=_probe_reducer)
    w = [1.0 / PROBE_K] * PROBE_K
    leg.ready()
    elapsed, kern_ms, _ = run_timed(_probe_step(lambda: agg.aggregate(w)), 1, a.steps, a.warmup, leg, False,
                                    False, sync=lambda: None, event=HostEvent)
    elapsed, achieved, hbm, _ = over_ranks(leg, elapsed, 0.0, 0.0, None)
    return {"mode": "param", "probe": True, "ms_per_step": elapsed / a.steps * 1e3}


def probe_client_axis(a, config: str, leg: Leg, dev) -> dict:
    rows = _probe_rows(PROBE_K // leg.world, 20 + leg.rank)
    agg = ClientAxisAggregator(rows, PROBE_N, chunks=2, reducer=_probe_reducer)
    w = [1.0 / PROBE_K] * rows.shape[0]
    steps, warmup = leg_steps(a)
    leg.ready()
    elapsed, _, _ = run_timed(_probe_step(lambda: agg.aggregate(w)), 1, steps, warmup, leg, False, False,
                              sync=lambda: None, event=HostEvent)
    elapsed, _, _, _ = over_ranks(leg, elapsed, 0.0, 0.0, None)
    return {"mode": "client", "probe": True, "backend": dist.get_backend(), "ms_per_step": elapsed / steps * 1e3}


def probe_inprocess(a, config: str, world: int) -> dict:
    rows = _probe_rows(PROBE_K, 30)
    out = torch.empty(PROBE_N)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        _probe_reducer(rows, [1.0 / PROBE_K] * PROBE_K, out)
    return {"mode": "one process", "probe": True, "devices": world,
            "ms_per_step": (time.perf_counter() - t0) / a.steps * 1e3}


# ---- the headline ---------------------------------------------------------------------------------------------------


def measure_headline(a, world: int, rank: int, dev, coord: Coord):
    """The line's own measurement (the contract's K timed steps).  Returns
    (line, the bucket and local sample counts for the CPU baseline)."""
    cfg = CONFIGS[a.config]
    entries = model_entries(a.config)
    n_elems = elements_per_client(entries)  # per client, the whole model
    mode = a.mode if world > 1 else "single"
    weak = a.weak and world > 1
    # this rank's clients: all of them (single / param axis) or its share (client axis)
    K_total, K_loc, first = plan_clients(a.config, world, rank, mode, a.clients_total, a.weak, a.clients)
    K = K_loc
    # the keys this rank reduces: all of them, or its whole-key shard (param axis)
    my_entries = entries
    if mode == "param":
        plan = multidev.shard_plan(entries, world)
        if len(plan) < world:
            raise SystemExit(f"{a.config} has data in {len(plan)} keys: too few for {world} ranks in --mode param")
        my_entries = plan[rank]

    from fedml_amd.synth import sample_nums
    ns_all = sample_nums(K_total, seed=1)
    ns_local = ns_all[first:first + K_loc]
    total_n = sum(ns_all)
    w_local = [n / total_n for n in ns_local]  # global weights of this rank's clients
    leg = Leg(coord, "headline")

    server = None
    sharded_opt = None
    if a.fedopt and mode == "client":
        bucket = ClientBucket(entries, K_loc, dev)  # integer buffers promoted into the fp32 row
        if set(bucket.groups) != {torch.float32}:
            raise SystemExit("--fedopt over several GPUs takes an fp32 model (integer buffers promoted)")
    elif a.fedopt:
        from collections import OrderedDict

        from fedml_amd.fedopt import FedOptServer

        init = OrderedDict((k, torch.zeros(s, dtype=d)) for k, s, d in my_entries)
        mine = {k for k, _, _ in my_entries}
        params = [p for p in shapes.param_names(entries) if p in mine]
        server = FedOptServer(init, params, K_loc, a.fedopt, 1.0, 0.9 if a.fedopt == "sgd" else 0.0, dev)
        bucket = server.bucket
    elif a.op in ("secagg", "lsa"):
        if world > 1:
            raise SystemExit("--op secagg / lsa is a 1-GPU measurement")
        # the model's elements as finite-field int64 rows (LightSecAgg's
        # transform_tensor_to_finite output), one group
        bucket = ClientBucket([(k, s, torch.int64) for k, s, _ in entries], K, dev, promote_ints=False)
    else:
        bucket = ClientBucket(my_entries, K_loc, dev, low_precision_acc=a.acc)
    for gi, (dt, g) in enumerate(bucket.groups.items()):
        if a.op in ("secagg", "lsa"):
            gen = torch.Generator(device=dev).manual_seed(1000 * rank + gi)
            g.rows.random_(0, LSA_PRIME, generator=gen)
        else:
            fill_rows(g.rows, g.length, seed=1000 * rank + gi, round_idx=3)
    torch.cuda.synchronize()

    groups = list(bucket.groups.items())
    dom_dt = max(groups, key=lambda kv: kv[1].length * kv[1].rows.element_size())[0]
    xgmi_bytes = 0

    # per-step work -------------------------------------------------------------
    if a.fedopt and mode == "client":
        from fedml_amd.sharded import ShardedFedOpt, buffer_ranges

        gd = bucket.groups[torch.float32]
        init = torch.zeros(gd.length, dtype=torch.float32, device=dev)
        sharded_opt = ShardedFedOpt(gd.rows, gd.length, init, a.fedopt, 1.0, 0.9 if a.fedopt == "sgd" else 0.0,
                                    chunks=a.chunks, buffers=buffer_ranges(bucket, shapes.param_names(entries)))

        def step(ev=None, cev=None):
            sharded_opt.aggregate(w_local, events=ev, comm_events=cev)

        n_launch = len(sharded_opt.agg.bounds)
        leg.ready()
        sharded_opt.aggregate(w_local)  # first step (no state read) before timing
        dom_bytes = K_loc * gd.length * 4 + gd.length * 4  # rows in, fp32 partial out (the step is 1/G of a pass)
        xgmi_bytes = (world - 1) * sharded_opt.agg.piece * len(sharded_opt.agg.bounds) * 4
    elif server is not None:
        for i, n in enumerate(ns_local):
            server.sample_num_dict[i] = n

        def step(ev=None, cev=None):
            server.aggregate(events=ev)

        n_launch = 1
        server.aggregate()  # first step (no momentum read) happens before timing
        dom_bytes = server.algorithmic_bytes()
    elif a.op == "median":
        from fedml_amd import defense as dfn

        if world > 1:
            raise SystemExit("--op median is a 1-GPU measurement")
        gd = bucket.groups[dom_dt]
        med_out = torch.empty(gd.padded, dtype=gd.rows.dtype, device=dev)  # the median is one of the inputs

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            dfn.median_rows(gd.d_ptrs, K, gd.length, med_out, aligned=True)
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = (K + 1) * gd.length * gd.rows.element_size()
    elif a.op == "rlr":
        # the robust-learning-rate defense: FedAvg chain + per-coordinate sign
        # sum + the lr rule, one pass over the fp32 row (threshold K/4)
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op rlr is a 1-GPU measurement")
        gd = bucket.groups[torch.float32]
        rlr_out = torch.empty(gd.padded, dtype=torch.float32, device=dev)
        rlr_w = kn.weights_for([n / sum(ns_local) for n in ns_local], torch.float32, dev)

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            kn.wsum_rlr_ptrs(gd.d_ptrs, rlr_w, K, gd.length, float(max(1, K // 4)), rlr_out, True)
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = (K + 1) * gd.length * 4
    elif a.op == "mpi":
        # the MPI simulation's term order (FedAVGAggregator.py:99-116) over the
        # dominant row: two roundings and a correctly rounded division per term
        from fedml_amd import _native as nat
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op mpi is a 1-GPU measurement")
        gd = bucket.groups[dom_dt]
        mpi_out = torch.empty(gd.padded, dtype=gd.out_dtype, device=dev)
        mpi_w = kn.muldiv_weights(dom_dt, [(n, sum(ns_local)) for n in ns_local], dev)
        code = kn._DT_CODE[dom_dt]
        call = lambda: nat.lib().fedagg_wsum_muldiv(  # noqa: E731
            code, gd.d_ptrs.data_ptr(), mpi_w.data_ptr(), K, gd.length, mpi_out.data_ptr(), nat.FEDAGG_ALIGNED16,
            nat.stream_handle())

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), "mpi")
            if ev is not None:
                ev[1].record()

        n_launch = 1
        dom_bytes = K * gd.length * gd.rows.element_size() + gd.length * torch.empty((), dtype=gd.out_dtype).element_size()
    elif a.op in ("krum", "dist2", "clip"):
        # the distance defenses' kernels over the fp32 row's weight keys
        # (csrc/robust.hip): krum = the K x K pair kernel, dist2 = every
        # client's distance to a global row, clip = the clipped rebuild
        from fedml_amd import _native as nat
        from fedml_amd import defense as dfn
        from fedml_amd import kernels as kn

        if world > 1:
            raise SystemExit("--op krum / dist2 / clip is a 1-GPU measurement")
        gd = bucket.groups[torch.float32]
        ref_row = gd.rows[K - 1].clone()  # a "global model" row
        if a.op == "krum":
            chunks, n_chunks = dfn.weight_chunks(gd, nat.PAIR_CHUNK, dev)
            pd_out = torch.empty((K, K), dtype=torch.float64, device=dev)
            gram = a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= dfn.GRAM_MAX_CLIENTS)
            work = dfn._work(nat.WORK_PAIRGRAM if gram else nat.WORK_PAIRDIST2, K, n_chunks, dev)
            pair_fn = nat.lib().fedagg_pairgram2_f32 if gram else nat.lib().fedagg_pairdist2_f32
            call = lambda: pair_fn(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, chunks.data_ptr(), n_chunks, pd_out.data_ptr(), work.data_ptr(),
                work.numel(), nat.stream_handle())
        elif a.op == "dist2":
            chunks, n_chunks = dfn.weight_chunks(gd, nat.DIST_CHUNK, dev)
            d_out = torch.empty(K, dtype=torch.float64, device=dev)
            work = dfn._work(nat.WORK_DIST2, K, n_chunks, dev)
            call = lambda: nat.lib().fedagg_dist2_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, ref_row.data_ptr(), chunks.data_ptr(), n_chunks, d_out.data_ptr(),
                work.data_ptr(), work.numel(), nat.stream_handle())
        else:
            clip_out = torch.empty_like(gd.rows)
            d_dst = kn.upload_i64([clip_out[i].data_ptr() for i in range(K)], dev)
            d_div = kn.upload_f32([1.0 + 0.01 * i for i in range(K)], dev)
            call = lambda: nat.lib().fedagg_clip_diff_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, ref_row.data_ptr(), d_div.data_ptr(), gd.length, d_dst.data_ptr(),
                nat.stream_handle())
        n_weight = sum(n for k, n in zip(gd.keys, gd.numels) if dfn.is_weight_param(k))
        gram = a.op == "krum" and (a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= 128))
        # krum, exact kernel: 3 flops (sub, mul, add) per client pair and weight element (VALU-bound);
        # krum, centred Gram on the bf16 matrix cores: the K weight rows read once (HBM-bound: its
        # six bf16 MFMAs per 32 columns need ~2/3 of the time the rows take to stream);
        # dist2: K rows + the reference row read once; clip: K rows in + K out + the reference row
        dom_bytes = {"krum": K * n_weight * 4 if a.op == "krum" and gram else 3 * K * (K - 1) // 2 * n_weight,
                     "dist2": (K + 1) * n_weight * 4, "clip": (2 * K + 1) * gd.length * 4}[a.op]
        krum_pair_flops = 2 * K * (K - 1) // 2 * n_weight  # one multiply-add per client pair and element

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), a.op)
            if ev is not None:
                ev[1].record()

        n_launch = 1
    elif a.op in ("secagg", "lsa"):
        from fedml_amd import _native as nat

        gd = bucket.groups[torch.int64]
        if a.op == "secagg":
            sec_out = torch.empty(gd.padded, dtype=torch.int64, device=dev)
            call = lambda: nat.lib().fedagg_sum_mod_i64(gd.d_ptrs.data_ptr(), K, gd.length, LSA_PRIME,  # noqa: E731
                                                        sec_out.data_ptr(), nat.FEDAGG_ALIGNED16, nat.stream_handle())
            dom_bytes = (K + 1) * gd.length * 8
        else:
            mask = torch.empty(gd.padded, dtype=torch.int64, device=dev).random_(0, LSA_PRIME)
            sec_out = torch.empty(gd.padded, dtype=torch.float32, device=dev)
            call = lambda: nat.lib().fedagg_lsa_reconstruct_f32(  # noqa: E731
                gd.d_ptrs.data_ptr(), K, gd.length, mask.data_ptr(), LSA_PRIME, LSA_QBITS, 1.0 / K,
                sec_out.data_ptr(), nat.FEDAGG_ALIGNED16, nat.stream_handle())
            dom_bytes = (K + 1) * gd.length * 8 + gd.length * 4

        def step(ev=None, cev=None):
            if ev is not None:
                ev[0].record()
            nat.check(call(), a.op)
            if ev is not None:
                ev[1].record()

        n_launch = 1
    elif mode in ("single", "param"):
        # one GPU, or this rank's whole-key shard of every client: the
        # single-GPU reduction over the bucket, no exchange
        outs = bucket.new_outputs()
        w = w_local if mode == "param" else bucket.weights(ns_local)

        def step(ev=None, cev=None):
            bucket.reduce_into(outs, w, events={dom_dt: ev} if ev is not None else None)

        n_launch = 1
        gd = bucket.groups[dom_dt]
        dom_bytes = K_loc * gd.length * gd.rows.element_size() + \
            gd.length * torch.empty((), dtype=gd.out_dtype).element_size()
    else:  # client axis: this rank's clients' partial + chunked RCCL reduce-scatter
        step, n_launch, dom_bytes, xgmi_bytes = client_axis_step(bucket, dom_dt, w_local, a.chunks, world)
        leg.ready()

    timed_comm = mode == "client" and world > 1 and a.backend == "nccl"
    elapsed, kern_ms, comm_ms = run_timed(step, n_launch, a.steps, a.warmup, leg, mode == "client", timed_comm)
    achieved = dom_bytes / (kern_ms / 1e3) / 1e9  # GB/s (GFLOP/s for the exact-difference krum kernel)
    hbm_all = dom_bytes / (elapsed / a.steps) / 1e9  # this rank's algorithmic bytes over the step time
    if world > 1:
        elapsed, achieved, hbm_all, comm_ms = over_ranks(leg, elapsed, achieved, hbm_all, comm_ms)

    ms_per_step = elapsed / a.steps * 1e3
    gram_op = a.op == "krum" and (a.pair_distance == "gram" or (a.pair_distance == "auto" and K <= 128))
    value = K_total * n_elems / (elapsed / a.steps)
    variant = a.fedopt or ("" if a.op == "fedavg" else a.op)
    if a.acc == "fp32" and dom_dt in (torch.bfloat16, torch.float16) and a.op == "fedavg":
        variant = (variant + "+" if variant else "") + "acc32"  # the fp32-accumulate kernel's own PMC entry
    traffic = load_traffic(a.config, mode, world, variant, K_loc)
    parallelism = {"single": "1 GPU",
                   "client": f"client-axis x{world}: {K_total} clients, ~{K_total // world} per GPU, fp32 partial + "
                             f"RCCL reduce-scatter, {a.chunks}-chunk pipeline",
                   "param": f"parameter-axis x{world}: every GPU holds its whole keys of all {K_total} clients "
                            f"(fedml_amd.multidev.shard_plan), no collective, bit-exact"}[mode]
    if weak:
        parallelism += f" [weak: {K} clients per GPU]"
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "client-params/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "int64" if a.op in ("secagg", "lsa") else "bf16" if dom_dt == torch.bfloat16 else "f32",
        "data": "synthetic (base~N(0,0.05^2), client=base+0.01*eps, generated in HBM)",
        "config": {
            "workload": cfg["desc"] + (f" [--clients {K}]" if a.clients is not None else ""),
            "clients_per_gpu": K_loc,
            "clients_total": K_total,
            "elements_per_client": n_elems,
            "layout": "ClientBucket rows [K, L] per dtype, 256-B aligned rows",
            "low_precision_acc": a.acc,
            "server_step": (SERVER_STEP_DESC[a.fedopt]
                            + (" fused" if server is not None else
                               f", on each rank's 1/{world} shard after the reduce-scatter, sharded state")
                            if a.fedopt else None),
            "parallelism": parallelism,
        },
        "roofline": {
            "bound": "valu" if a.op == "krum" and not gram_op else "hbm",
            "achieved": round(achieved / 1e3, 2) if a.op == "krum" and not gram_op else round(achieved, 1),
            "peak": VALU_PEAK_TFLOPS if a.op == "krum" and not gram_op else HBM_PEAK_GBPS,
            "unit": "TFLOP/s" if a.op == "krum" and not gram_op else "GB/s",
            "frac": round(achieved / 1e3 / VALU_PEAK_TFLOPS if a.op == "krum" and not gram_op
                          else achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "kernel": ({"secagg": "reduce_kernel<OpSumModI64>", "lsa": "reduce_kernel<OpWrapSumI64, LsaEpi>",
                        "krum": ((f"pairgram_split8_kernel<{(K + 15) // 16}> + gram_sum_kernel + gram_dist_kernel "
                                  "(centred Gram, exact 3-way bf16 split, 16x16x32 bf16 MFMA)") if a.pair_distance == "gram" or
                                 (a.pair_distance == "auto" and K <= 128) else
                                 ("pairtri_kernel<16> + tri_finish_kernel" if K <= 64 else
                                  "pairtri_kernel<32> + tri_finish_kernel" if K <= 128 else
                                  "pairdist_kernel + pair_finish_kernel") + " (packed fp32)"),
                        "dist2": "dist2_kernel + sum_rows_kernel",
                        "clip": "clip_diff_kernel", "rlr": "reduce_kernel<OpF32Rlr, RlrEpi>",
                        "mpi": "reduce_kernel<OpF32MulDiv> (fl(fl(p n_i) / N))"}[a.op]
                       if a.op in ("secagg", "lsa", "krum", "dist2", "clip", "rlr", "mpi") else
                       median_kernel_name(K, dom_dt) if a.op == "median" else
                       SERVER_STEP_KERNEL.get(a.fedopt, "reduce_kernel<OpF32,SgdEpi>") + " (FedAvg+server step fused)"
                       if server is not None else
                       f"reduce_kernel<OpF32> x{n_launch}/step + shard step" if sharded_opt is not None else
                       f"reduce_kernel<{'OpF32' if dom_dt == torch.float32 else dom_dt}> x{n_launch}/step"),
            "alg_bytes_per_step": dom_bytes,
            "kernel_ms_per_step": round(kern_ms, 4),
            **({"useful_tflops": round(krum_pair_flops / (kern_ms / 1e3) / 1e12, 2),
                # NT 16x16 tiles x 12 MFMAs of 16 cycles per 64 columns, over 1024 SIMDs at 2.4 GHz
                "bf16_mfma_floor_ms": round(((K + 15) // 16) * ((K + 15) // 16 + 1) // 2 * 12 * 16 * (n_weight / 64)
                                            / (1024 * 2.4e9) * 1e3, 3)}
               if gram_op else {}),
        },
        "cpu_baseline": None,
    }
    if a.op == "median":
        # the sorting networks are VALU-bound above ~128 clients: their min / max /
        # med3 / DPP ops issue at 4 cycles per wave64 instruction per SIMD
        # (tools/valu_rate_probe.hip), so this is the share of the SIMDs' issue
        # capacity the kernel's executed VALU instructions take
        vv = load_median_valu(a.config, mode, world, variant, K_loc)
        if vv:
            issue_ms = vv["valu_instr_per_wave"] * vv["waves_per_launch"] * VALU_HALF_RATE_CYCLES / (
                SIMDS * CLOCK_GHZ * 1e9) * 1e3
            line["roofline"]["valu"] = {
                "bound": "valu issue (half-rate ops, 4 cycles per wave64 instruction per SIMD)",
                "instr_per_wave": vv["valu_instr_per_wave"], "waves_per_launch": vv["waves_per_launch"],
                "issue_ms_at_peak": round(issue_ms, 4), "frac": round(issue_ms / kern_ms, 4),
                "source": "profiles/median_valu.json (SQ_INSTS_VALU / SQ_WAVES)"}
    if world > 1:
        # whole-job HBM rate: every rank's algorithmic bytes over the step time
        line["roofline"]["aggregate_gbps"] = round(hbm_all, 1)
        line["roofline"]["aggregate_frac_of_n_peaks"] = round(hbm_all / (world * HBM_PEAK_GBPS), 4)
        if mode == "client":
            line["exchange"] = {"mode": "client", "backend": dist.get_backend(), "world_size": world,
                                "collective": "reduce_scatter_tensor (RCCL)" if a.backend == "nccl" else "gloo (host)",
                                "xgmi_bytes_per_rank_per_step": xgmi_bytes,
                                "comm_ms_per_step": round(comm_ms, 4) if comm_ms is not None else None,
                                "note": "comm_ms: mean over ranks of the chunks' reduce-scatter time on the comm "
                                        "stream (overlapping the next chunk's reduction)"}
    keep = (bucket, ns_local) if world == 1 and a.op == "fedavg" and not a.no_cpu_baseline else None
    return line, keep


SERVER_STEP_DESC = {"sgd": "SGD lr=1.0 momentum=0.9", "adam": "Adam lr=1.0 betas=(0.9,0.999)",
                    "adagrad": "Adagrad lr=1.0 eps=1e-10", "adamw": "AdamW lr=1.0 weight_decay=0.01",
                    "rmsprop": "RMSprop lr=1.0 alpha=0.99", "adamax": "Adamax lr=1.0 betas=(0.9,0.999)",
                    "nadam": "NAdam lr=1.0 momentum_decay=4e-3", "radam": "RAdam lr=1.0 betas=(0.9,0.999)",
                    "adadelta": "Adadelta lr=1.0 rho=0.9 eps=1e-6", "asgd": "ASGD lr=1.0 lambd=1e-4 alpha=0.75",
                    "rprop": "Rprop lr=1.0 etas=(0.5,1.2)"}
SERVER_STEP_KERNEL = {"adam": "reduce_fused_kernel<OpF32,AdamEpi>", "adamw": "reduce_fused_kernel<OpF32,AdamEpi>",
                      "adagrad": "reduce_kernel<OpF32,AdagradEpi>", "rmsprop": "reduce_kernel<OpF32,AdagradEpi>",
                      **{o: f"reduce_fused_kernel<OpF32,OptRepoEpi<{c}>>" for o, c in
                         (("adamax", 1), ("nadam", 2), ("radam", 3), ("adadelta", 4), ("asgd", 5), ("rprop", 6))}}


def probe_headline(a, world: int, rank: int, coord: Coord):
    """--probe-cpu: the multi-rank orchestration with a host stand-in for the
    parameter-axis reduction (gloo, no GPU).  Not a measurement."""
    d = probe_param(a, a.config, Leg(coord, "headline"), None)
    line = {"metric": METRIC, "value": PROBE_K * PROBE_N / (d["ms_per_step"] / 1e3), "unit": "client-params/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": d["ms_per_step"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "probe", "probe": "cpu orchestration probe: host stand-in reductions over gloo, not a measurement",
            "config": {"workload": "probe", "parallelism": f"parameter-axis x{world}"}, "roofline": None,
            "cpu_baseline": None}
    return line, None


def nested_configs(a, world: int):
    """The config legs nested in this run (--nest, default by N)."""
    if a.nest == "none":
        return []
    if a.nest == "auto":
        want = (["cfg4"] if world >= 4 else []) + (["cfg5"] if world >= 8 else [])
    else:
        want = [c.strip() for c in a.nest.split(",") if c.strip()]
        bad = [c for c in want if c not in ("cfg4", "cfg5")]
        if bad:
            raise SystemExit(f"--nest: {bad} (cfg4 / cfg5, auto or none)")
    return [c for c in want if c != a.config]


def run_nested(a, world: int, rank: int, dev, coord: Coord, budget: Budget, line: dict) -> None:
    """The nested legs of a multi-GPU --mode param FedAvg line, each into its
    own object of ``line`` (which the watchdog prints as it stands)."""
    probe = a.probe_cpu
    cleanup = (lambda: None) if probe else _free_device_memory
    client_fn = probe_client_axis if probe else measure_client_axis
    inproc_fn = probe_inprocess if probe else measure_inprocess
    param_fn = probe_param if probe else measure_param
    sfo_fn = probe_client_axis if probe else measure_sharded_fedopt
    ifo_fn = probe_inprocess if probe else measure_inprocess_fedopt

    def leg(key, name, fn, rank0_only=False):
        res = run_leg(coord, budget, name, fn, LEG_RESERVE_S.get(name, 45.0), rank0_only, cleanup)
        tgt = line
        for part in key[:-1]:
            tgt = tgt.setdefault(part, {})
        tgt[key[-1]] = res

    cleanup()
    if not a.no_exchange:
        leg(("exchange",), "exchange", lambda lg: client_fn(a, a.config, lg, dev))
    if not a.no_inprocess:
        leg(("inprocess",), "inprocess", lambda lg: inproc_fn(a, a.config, world), rank0_only=True)
    for cfg in nested_configs(a, world):
        if cfg == "cfg4":
            leg(("cfg4", "param"), "cfg4/param", lambda lg: param_fn(a, "cfg4", lg, dev))
            if not a.no_exchange:
                leg(("cfg4", "exchange"), "cfg4/exchange", lambda lg: client_fn(a, "cfg4", lg, dev))
            if not a.no_inprocess:
                leg(("cfg4", "inprocess"), "cfg4/inprocess", lambda lg: inproc_fn(a, "cfg4", world), rank0_only=True)
        elif cfg == "cfg5":
            if not a.no_exchange:
                leg(("cfg5", "sharded_fedopt"), "cfg5/sharded_fedopt", lambda lg: sfo_fn(a, "cfg5", lg, dev))
            if not a.no_inprocess:
                leg(("cfg5", "inprocess_fedopt"), "cfg5/inprocess_fedopt", lambda lg: ifo_fn(a, "cfg5", world),
                    rank0_only=True)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched as `python bench.py --gpus N`: become torchrun ourselves
        raise SystemExit(spawn_ranks(a.gpus, sys.argv[1:], probe=a.spawn_probe))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus > 1 and world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one process per GPU (or drop WORLD_SIZE "
                         "and let bench.py spawn them)")
    if a.spawn_probe:
        print(json.dumps({"probe": "rank", "rank": rank, "local_rank": local, "world": world,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}",
                          "cuda_initialized": torch.cuda.is_initialized()}), flush=True)
        return
    budget = Budget(a.budget_s)
    dev = None
    if not a.probe_cpu:
        dev = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    coord = SOLO
    if world > 1:
        start_watchdog(rank, budget, a.watchdog_s)
        timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
        # no device_id: RCCL builds its communicator at the first collective
        # (a nested client-axis leg), so the exchange-free headline needs only
        # the rendezvous store
        backend = "gloo" if a.probe_cpu or a.backend == "gloo" else "nccl"
        dist.init_process_group(backend, timeout=timeout)
        coord = Coord(world, rank, dist.distributed_c10d._get_default_store())
    keep = None
    try:
        if a.probe_cpu:
            if world == 1:
                raise SystemExit("--probe-cpu rehearses the multi-rank orchestration: --gpus >= 2")
            line, keep = probe_headline(a, world, rank, coord)
        else:
            line, keep = measure_headline(a, world, rank, dev, coord)
        if rank == 0:
            REPORT.line = line
        if world > 1 and a.mode == "param" and a.op == "fedavg" and not a.fedopt:
            try:
                run_nested(a, world, rank, dev, coord, budget, line)
            except Exception as e:  # noqa: BLE001 -- the headline stands whatever the nested legs hit
                line["nested_error"] = f"{type(e).__name__}: {e}"
        if keep is not None and rank == 0:  # the reference's FedAvg loop on the host
            line["cpu_baseline"] = cpu_baseline(keep[0], keep[1], a.cpu_reps)
        REPORT.emit()
    finally:
        if world > 1 and dist.is_initialized():
            try:
                coord.barrier("exit", timeout_s=30.0)
            except (TimeoutError, RuntimeError):
                pass
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
