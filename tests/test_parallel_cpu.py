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


def _objects():
    import synthetic as S

    objs = []
    for i in range(5):
        o = S.make_object(500 + i, n_pts=40 + 13 * i, n_bg=10 + 7 * i, scale=1.0, tz=3.0, upright=False)
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
