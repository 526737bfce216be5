"""bench.py's self-launch (CPU): `python bench.py --gpus N` without torchrun
spawns N ranks with torchrun's environment, and the parent never initialises
HIP (a process that has touched the GPU must not start the ranks; they are
fresh processes, not forks)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=e, cwd=ROOT)


def test_spawn_gives_every_rank_torchrun_env_and_parent_stays_off_the_gpu():
    p = _run(["--gpus", "3", "--backend", "gloo", "--spawn-probe"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    ranks = sorted((d for d in lines if d["probe"] == "rank"), key=lambda d: d["rank"])
    parent = [d for d in lines if d["probe"] == "parent"]
    assert [d["rank"] for d in ranks] == [0, 1, 2]
    assert all(d["world"] == 3 and d["local_rank"] == d["rank"] for d in ranks)
    assert len({d["master"] for d in ranks}) == 1 and ranks[0]["master"].startswith("127.0.0.1:")
    assert not any(d["cuda_initialized"] for d in ranks)
    assert parent == [{"probe": "parent", "cuda_initialized": False, "exit_codes": [0, 0, 0]}]


def test_spawn_propagates_a_failing_rank():
    """A rank that dies ends the launch with its exit code (here: no GPU in
    this container, so every real rank fails before its first collective)."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "2"], env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


def _barrier_rank(rank, world, port, out):
    import time as _t

    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    t0 = _t.perf_counter()
    if rank == 1:
        _t.sleep(0.5)
    bench.host_barrier("t1", world)
    waited = _t.perf_counter() - t0
    bench.host_barrier("t2", world)  # a second barrier with its own tag
    out.put((rank, waited))
    dist.destroy_process_group()


def test_host_barrier_waits_for_every_rank():
    """bench.host_barrier (the TCP-store barrier around the one-process
    measurement): rank 0 leaves only after the late rank 1 arrives."""
    import torch.multiprocessing as mp

    sys.path.insert(0, ROOT)
    import bench

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_barrier_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert got[0] >= 0.45 and all(p.exitcode == 0 for p in ps)
