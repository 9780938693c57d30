"""bench.py's multi-GPU plumbing (replicas only) rehearsed on CPU with gloo,
world_size 2: process-group init from the torchrun environment, the barrier, and the
aggregate = (max seconds over ranks, sum of tokens over ranks) that `value` is built from."""
import os
import socket
import sys
from pathlib import Path

import torch
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(ws), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    import bench

    r, w, lr = bench.dist_init()
    bench.barrier(w)
    t, n = bench.aggregate(0.5 + rank, 100 * (rank + 1), w)
    q.put((r, w, lr, t, n))
    import torch.distributed as dist

    dist.destroy_process_group()


def test_replica_aggregate_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[:3] for r in res] == [(0, 2, 0), (1, 2, 1)]
    for _, _, _, t, n in res:
        assert t == 1.5 and n == 300  # max of (0.5, 1.5); 100 + 200 tokens


def test_single_process_is_identity():
    sys.path.insert(0, str(REPO))
    import bench

    assert bench.aggregate(2.0, 7, 1) == (2.0, 7)
    assert not torch.distributed.is_initialized()


def test_bench_spawns_its_own_replicas():
    """`bench.py --gpus 2` started WITHOUT a launcher spawns one replica process per GPU with
    the torchrun environment (the driver's SCALE runs and C4 rely on it); --stub replaces the
    GPU work so the launch / barrier / aggregation path runs here on CPU with gloo."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--stub", "--steps", "3",
                          "--warmup", "1"], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["stub"] is True and line["steps"] == 3
    assert line["value"] > 0


def test_bench_replica_failure_stops_siblings():
    """One replica dying (here rank 1 exits 3 before the barrier) must not leave rank 0 blocked in
    the gloo barrier until the driver's time limit: the launcher polls every child, terminates the
    others on the first non-zero exit and returns that exit code (advisor finding, round 2)."""
    import subprocess
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--stub", "--stub-fail-rank", "1",
                          "--steps", "3", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    took = time.monotonic() - t0
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert "stopping the others" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert took < 120, took  # gloo's own barrier timeout is 30 min
