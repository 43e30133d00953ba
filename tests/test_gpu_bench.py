"""bench.py's multi-rank path on one GPU (the driver's N>1 runs use RCCL over xGMI, one GPU
per rank; here two gloo ranks share device 0, which RCCL refuses).

``python bench.py --gpus 2`` with no launcher starts torch.distributed.run itself; each rank
uploads its LPT shard (reconstruct/parallel.py: ResidentShard), and one all-gather returns
every object's record to rank 0.  The gathered records must be bitwise those of a
one-process run of the same job — objects never interact, and a batch's
results do not depend on how the objects are split into batches (test_batch_equals_single).
This replaces the reference's sequential per-detection loop
(/root/reference/src/LocalMapping_util.cc:165-206) with object-sharded ranks.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


ARGS = ["--steps", "1", "--warmup", "0", "--objects", "8", "--no-extra", "--no-cpu-baseline", "--no-config4"]


def _bench(n, dump, extra=(), env_extra=None, launcher=()):
    env = dict(os.environ, DSR_BENCH_BACKEND="gloo")
    env.update(env_extra or {})
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, *launcher, "bench.py", "--gpus", str(n), *ARGS, "--dump-records", dump, *extra]
    p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n", [2, 4])
def test_bench_two_ranks_gather_equals_one_process(tmp_path, n):
    """n gloo ranks on device 0 (4: the 2-objects-per-rank shards of an 8-object job)."""
    two = _bench(n, str(tmp_path / "two.npy"))
    one = _bench(1, str(tmp_path / "one.npy"))
    assert two["n_gpus"] == n and one["n_gpus"] == 1
    r = two["ranks"]
    assert r["world_size_observed"] == n and r["backend"] == "gloo" and len(r["rank_seconds"]) == n
    assert sorted(r["shard_objects"]) == [8 // n] * n and r["gather_ms_per_step"] > 0
    assert two["config"]["objects"] == one["config"]["objects"] == 8
    a, b = np.load(tmp_path / "two.npy"), np.load(tmp_path / "one.npy")
    assert a.shape == b.shape == (8, 83)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a[:, 1] == 1).all()
    assert two["lite_broken_blocks"] == 0 == one["lite_broken_blocks"]


@pytest.mark.timeout(300)
def test_bench_rccl_path_on_one_rank(tmp_path):
    """The driver's N>1 runs go through torch.distributed.run with backend "nccl" (RCCL over
    xGMI), which needs one GPU per rank.  On this one-GPU box the same code path runs with one
    rank (DSR_BENCH_FORCE_DIST=1): RCCL process group, device-tensor all-gather of the records,
    barrier and max-over-ranks timing — records bitwise those of the plain one-process run."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    launcher = ("-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr", "127.0.0.1",
                "--master-port", str(port))
    rccl = _bench(1, str(tmp_path / "rccl.npy"), env_extra={"DSR_BENCH_FORCE_DIST": "1", "DSR_BENCH_BACKEND": "nccl"},
                  launcher=launcher)
    one = _bench(1, str(tmp_path / "one.npy"))
    r = rccl["ranks"]
    assert r["backend"] == "nccl" and r["world_size_observed"] == 1 and r["gather_ms_per_step"] > 0
    assert "backend" not in one["ranks"]
    a, b = np.load(tmp_path / "rccl.npy"), np.load(tmp_path / "one.npy")
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.timeout(600)
def test_bench_eight_ranks_rehearse_the_driver_command(tmp_path):
    """The driver's N = 8 command, rehearsed on one GPU: ``bench.py --gpus
    8`` with no launcher spawns 8 ranks (gloo, all on device 0 — RCCL needs a GPU per rank),
    each uploads its LPT shard of a 16-object job and of the config-4 leg (64 objects x 1024
    points here, 8 per rank as at N = 8), one all-gather returns every record to rank 0 — and
    both record sets are bitwise those of ``--gpus 1``."""
    extra = ["--objects", "16", "--c4-objects", "64", "--c4-pts", "1024"]
    args8 = [a for a in ARGS if a not in ("--no-config4",)]

    def run(n, dump):
        env = dict(os.environ, DSR_BENCH_BACKEND="gloo")
        env.pop("WORLD_SIZE", None)
        cmd = [sys.executable, "bench.py", "--gpus", str(n), *args8, *extra, "--dump-records", dump]
        p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=500)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads(p.stdout.strip().splitlines()[-1])

    eight = run(8, str(tmp_path / "eight.npy"))
    one = run(1, str(tmp_path / "one.npy"))
    r = eight["ranks"]
    assert eight["n_gpus"] == 8 and r["world_size_observed"] == 8 and r["backend"] == "gloo"
    assert len(r["rank_seconds"]) == 8 and sorted(r["shard_objects"]) == [2] * 8
    assert eight["config4"]["shard_objects"] == [8] * 8 and one["config4"]["shard_objects"] == [64]
    for name in ("eight", "eight_c4"):
        a, b = np.load(tmp_path / f"{name}.npy"), np.load(tmp_path / f"{name.replace('eight', 'one')}.npy")
        assert a.shape == b.shape and a.shape[0] in (16, 64)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), name
        assert (a[:, 1] == 1).all()
