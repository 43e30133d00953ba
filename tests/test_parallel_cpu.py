"""Multi-rank object sharding (reconstruct/parallel.py) on CPU with gloo, world_size 2.

The per-rank solver is injected: here the CPU oracle on tiny objects (test
infrastructure); on GPUs it is Optimizer.reconstruct_objects over RCCL.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _objects(n=5, ragged=True):
    import synthetic as S

    objs = []
    for i in range(n):
        k = i if ragged else 0
        o = S.make_object(500 + i, n_pts=40 + 13 * k, n_bg=10 + 7 * k, scale=1.0, tz=3.0, upright=False)
        objs.append((o.t_cam_obj, o.pts, o.rays, o.depth, None))
    return objs


def _solver():
    from deep_sdf.workspace import fold_state

    import synthetic as S
    from oracle import dsr_oracle as O

    dec = O.Decoder(fold_state(S.make_decoder(1234), S.DEFAULT_SPECS))
    P = O.OptimParams.from_cfg(dict(S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"],
                                                                      num_iterations=1)))

    def solve(objs):
        out = []
        for t, p, r, d, c in objs:
            res = O.reconstruct_object(dec, P, t, p, r, d, c)
            out.append({"t_cam_obj": res.t_cam_obj, "code": res.code, "is_good": res.is_good,
                        "loss": res.loss, "iters_done": len(res.trace)})
        return out

    return solve


def _worker(rank, world, port, q):
    import sys

    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from reconstruct.parallel import reconstruct_sharded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = reconstruct_sharded(_objects(), _solver())
        if rank == 0:
            q.put([(r["is_good"], r["loss"], None if r["t_cam_obj"] is None else r["t_cam_obj"].tolist(),
                    r["iters_done"]) for r in res])
    finally:
        dist.destroy_process_group()


class _FakeLib:
    """Stands in for libdsr's resident-batch entry points on CPU (test infrastructure): the
    batch keeps the objects dsr_batch_create received through the C structs and a run solves
    them with the CPU oracle, so ResidentShard's partition, upload, download, record packing
    and gather run exactly as on the GPU."""

    def __init__(self):
        self.batches = {}
        self.solve = _solver()

    def dsr_batch_create(self, ctx, dec, params, n, ins, hout):
        objs = []
        for k in range(n):
            r = ins[k]
            arr = lambda p, m: np.ctypeslib.as_array(p, shape=(m,)).copy()  # noqa: E731
            objs.append((np.array(r.t_cam_obj, np.float32).reshape(4, 4),
                         arr(r.pts, 3 * r.n_pts).reshape(-1, 3), arr(r.rays, 3 * r.n_rays).reshape(-1, 3),
                         arr(r.depth, r.n_depth), None))
        key = len(self.batches) + 1
        self.batches[key] = {"objs": objs, "res": None}
        hout._obj.value = key
        return 0

    def dsr_batch_run(self, h):
        b = self.batches[h.value]
        b["res"] = self.solve(b["objs"])
        return 0

    def dsr_batch_download(self, h, outs):
        for k, r in enumerate(self.batches[h.value]["res"]):
            o = outs[k]
            o.is_good = int(r["is_good"])
            o.loss = float(r["loss"])
            o.iters_done = int(r["iters_done"])
            if r["is_good"]:
                o.t_cam_obj[:] = np.asarray(r["t_cam_obj"], np.float32).reshape(-1).tolist()
                o.code[:] = np.asarray(r["code"], np.float32).tolist()
        return 0

    def dsr_batch_destroy(self, h):
        self.batches.pop(h.value, None)
        return 0


def _fake_optimizer():
    import ctypes

    import synthetic as S
    from reconstruct.optimizer import Optimizer
    from reconstruct.utils import ForceKeyErrorDict

    class Ctx:
        lib = _FakeLib()
        handle = ctypes.c_void_p(1)

        def check(self, rc, what):
            assert rc == 0, what

    class Dec:
        ctx = Ctx()
        handle = ctypes.c_void_p(2)

    cfg = ForceKeyErrorDict(data_type="Redwood", optimizer=dict(
        S.REDWOOD_OPTIM, joint_optim=dict(S.REDWOOD_OPTIM["joint_optim"], num_iterations=1)))
    return Optimizer(Dec(), cfg)


def _resident_worker(rank, world, port, q, n_obj=5):
    import sys

    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from reconstruct.parallel import ResidentShard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = ResidentShard(_fake_optimizer(), _objects(n_obj, ragged=n_obj == 5))
        first = shard.run()
        second = shard.run()                 # inputs stay resident: a re-run gives the same records
        shard.launch()                       # bench.py's overlapped steps: step s+1 launched
        shard.download()                     # before step s's records are packed and gathered
        shard.launch()
        third = shard.finish()
        shard.download()
        fourth = shard.finish()
        if rank == 0:
            q.put({"mine": shard.mine, "shards": shard.shards, "gather": shard.last_gather_s,
                   "res": [(r["is_good"], r["loss"], None if r["t_cam_obj"] is None else r["t_cam_obj"].tolist(),
                            r["iters_done"]) for r in first],
                   "same": all(a["loss"] == b["loss"] == c["loss"] == d["loss"]
                               for a, b, c, d in zip(first, second, third, fourth))})
        else:
            assert first is None and second is None and third is None and fourth is None
        shard.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_resident_shard_world2_equals_one_process():
    """bench.py's N>1 path (reconstruct/parallel.py: ResidentShard): each of 2 gloo ranks
    uploads only its LPT shard, runs it, and one all-gather returns every object's record to
    rank 0 in input order — equal to the one-process ResidentShard."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resident_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from reconstruct.parallel import ResidentShard

    one = ResidentShard(_fake_optimizer(), _objects())
    ref = one.run()
    assert sorted(i for s in got["shards"] for i in s) == list(range(len(ref)))
    assert all(len(s) > 0 for s in got["shards"]) and got["gather"] > 0.0 and got["same"]
    for (good, loss, T, it), r in zip(got["res"], ref):
        assert good == r["is_good"] and it == r["iters_done"]
        assert np.float32(loss) == np.float32(r["loss"])
        if good:
            assert np.array_equal(np.asarray(T, np.float32), np.asarray(r["t_cam_obj"], np.float32))


@pytest.mark.timeout(600)
def test_resident_shard_world8_equals_one_process(monkeypatch):
    """The driver's N = 8 path on CPU: 8 gloo ranks, one 64-object job of
    equal-cost objects — LPT gives every rank 8 (BASELINE config 4's split) — each rank uploads
    and runs only its shard, one all-gather returns every record to rank 0 in input order,
    bitwise the one-process ResidentShard's."""
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        monkeypatch.setenv(k, "1")          # 8 ranks on this host's cores: one BLAS thread each
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resident_worker, args=(r, 8, port, q, 64)) for r in range(8)]
    for p in procs:
        p.start()
    got = q.get(timeout=500)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from reconstruct.parallel import ResidentShard

    from threadpoolctl import threadpool_limits

    with threadpool_limits(1):              # the ranks' BLAS summation order (one thread each)
        ref = ResidentShard(_fake_optimizer(), _objects(64, ragged=False)).run()
    assert [len(s) for s in got["shards"]] == [8] * 8 and len(got["mine"]) == 8
    assert sorted(i for s in got["shards"] for i in s) == list(range(64))
    assert got["same"] and got["gather"] > 0.0
    assert len(got["res"]) == len(ref) == 64
    for (good, loss, T, it), r in zip(got["res"], ref):
        assert good == r["is_good"] and it == r["iters_done"]
        assert np.float32(loss) == np.float32(r["loss"])
        if good:
            assert np.array_equal(np.asarray(T, np.float32), np.asarray(r["t_cam_obj"], np.float32))


def test_bench_spawns_its_own_ranks(monkeypatch):
    """`python bench.py --gpus N` without a launcher starts torch.distributed.run with N local
    ranks as a child process (no exec of a process that touched the GPU)."""
    import subprocess
    import sys

    sys.path.insert(0, REPO)
    import bench

    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    (cmd,) = calls
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()
    # under a launcher WITHOUT --gpus (torchrun --nproc-per-node 8 bench.py): the launcher's ranks
    # are taken; only an explicit, disagreeing --gpus is an error
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "2"])
    monkeypatch.setenv("WORLD_SIZE", "2")
    args, world = bench.parse_args()
    assert args.gpus == 2 == world


def test_lpt_partition_balances_and_covers():
    from reconstruct.parallel import lpt_partition

    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    shards = lpt_partition(costs, 3)
    assert sorted(i for s in shards for i in s) == list(range(10))
    loads = [sum(costs[i] for i in s) for s in shards]
    assert max(loads) - min(loads) <= max(costs)
    assert lpt_partition([1, 2], 4)[2:] == [[], []]


@pytest.mark.timeout(300)
def test_sharded_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _solver()(_objects())
    assert len(got) == len(ref)
    for (good, loss, T, it), r in zip(got, ref):
        assert good == r["is_good"]
        assert np.float32(loss) == np.float32(r["loss"])
        assert it == r["iters_done"]
        if good:
            assert np.array_equal(np.asarray(T, np.float32), np.asarray(r["t_cam_obj"], np.float32))


@pytest.mark.parametrize("world", [1, 2, 8])
def test_rank_r_binds_device_r(world, monkeypatch):
    """at N = 8 rank r runs on HIP device r — bench.py binds it through
    parallel.rank_device (and exports it as DSR_DEVICE), the library's Context.get() default
    reads DSR_DEVICE / LOCAL_RANK — and an RCCL launch on a node with fewer visible devices than
    ranks exits with a message instead of running its ranks on device 0 (device count mocked)."""
    from reconstruct import _libdsr as L
    from reconstruct.parallel import rank_device

    for r in range(world):
        assert rank_device(r, world, "nccl", 8) == r
        assert rank_device(r, world, "gloo", 1) == 0          # CPU rehearsals share device 0
    if world > 1:
        with pytest.raises(RuntimeError, match="one GPU per rank"):
            rank_device(world - 1, world, "nccl", world - 1)
    with pytest.raises(RuntimeError):
        rank_device(world, world, "nccl", 8)

    made = []

    def fake_init(self, device=0):
        self.device = device
        self.handle = None
        made.append(device)

    monkeypatch.setattr(L.Context, "__init__", fake_init)
    monkeypatch.setattr(L.Context, "_cache", {})
    monkeypatch.delenv("DSR_DEVICE", raising=False)
    for r in range(world):
        monkeypatch.setenv("LOCAL_RANK", str(r))
        assert L.Context.get().device == r
        monkeypatch.setenv("DSR_DEVICE", str(r))               # what bench.py exports after binding
        assert L.Context.get().device == r
        monkeypatch.delenv("DSR_DEVICE")
    assert made == list(range(world))


def test_bench_binds_through_rank_device():
    """bench.py routes its rank -> device binding through parallel.rank_device (the checked
    helper above) before any process group or context exists, and records every rank's device."""
    src = open(os.path.join(REPO, "bench.py")).read()
    i_bind = src.index("local = rank_device(")
    assert i_bind < src.index("torch.cuda.set_device(local)") < src.index('dist.init_process_group("nccl"')
    assert 'os.environ["DSR_DEVICE"] = str(local)' in src
    assert "all_gather_object(devs, me)" in src and "distinct_devices" in src
