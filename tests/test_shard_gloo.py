"""Row-sharded frame assembly across processes on CPU (gloo): the product's
ShardPlan + gather_to_root (raymarching_amd/frame.py) with the oracle as the
per-rank renderer, checked bit for bit against a one-process frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import raymarching_amd as rm
from raymarching_amd.frame import ShardPlan, gather_parts_to_root, gather_to_root

W, H = 40, 37
POSE = rm.POSES["P2"]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, band, scene, q):
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan(W, H, band, world)
    rows = plan.rows(rank)
    local = torch.zeros((plan.rows_per_shard, W, 4), dtype=torch.float32)
    if rows:
        img, _ = oracle.render_rows(scene, W, H, rows, pos=POSE["pos"], mouse=POSE["mouse"], time=POSE["time"])
        local[: len(rows)] = torch.from_numpy(img)
    g = gather_to_root(local, plan, rank)
    if rank == 0:
        flat = g.reshape(world * plan.rows_per_shard, W, 4)
        frame = flat[plan.gathered_index()].numpy()
        q.put(frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 16), (3, 5), (2, 1)])
def test_gloo_sharded_frame_equals_single_process(world, band):
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, band, "O", q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = oracle.render("O", W, H, pos=POSE["pos"], mouse=POSE["mouse"], time=POSE["time"])
    np.testing.assert_array_equal(frame, full)


def weighted_worker(rank, world, port, runs, scene, q):
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan(W, H, runs[-1], world, runs)
    rows = plan.rows(rank)
    local = torch.zeros((len(rows), W, 4), dtype=torch.float32)
    if rows:
        pz = rm.S0_POSE
        img, _ = oracle.render_rows(scene, W, H, rows, pos=pz["pos"], mouse=pz["mouse"], time=pz["time"])
        local[:] = torch.from_numpy(img)
    out = None
    if rank == 0:
        out = torch.full((H, W, 4), float("nan"))
        out[: len(rows)] = local  # the root's rows are in place before the gather
    g = gather_parts_to_root(local, plan, rank, out=out)
    if rank == 0:
        q.put(g[plan.packed_index()].numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("runs", [(9, 4), (3, 5, 2), (40, 1), (1, 1, 1, 7)])
def test_gloo_weighted_parts_equal_single_process(runs):
    """Weighted cyclic parts (the balanced multi-GPU split): unpadded
    point-to-point gather, frame rebuilt through ShardPlan.packed_index."""
    import oracle
    world = len(runs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=weighted_worker, args=(r, world, port, runs, "S0", q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = oracle.render("S0", W, H, pos=rm.S0_POSE["pos"], mouse=rm.S0_POSE["mouse"], time=rm.S0_POSE["time"])
    np.testing.assert_array_equal(frame, full)


@pytest.mark.parametrize("H_,runs", [(37, (9, 4)), (4096, (26, 16)), (1080, (5, 27, 27, 27)), (9, (4, 4, 4, 4, 4)),
                                     (4096, (40,) + (16,) * 7)])
def test_weighted_plan_matches_c_abi(H_, runs):
    n = len(runs)
    plan = ShardPlan(8, H_, 16, n, runs)
    assert sum(plan.count(s) for s in range(n)) == H_
    for s in range(n):
        assert plan.count(s) == rm.cycle_rows(H_, plan.cycle, plan.offsets[s], runs[s]) == len(plan.rows(s))
    idx = plan.packed_index()
    assert sorted(idx) == list(range(H_))
    for y in range(0, H_, max(1, H_ // 50)):
        s, j = plan.slot_of_row(y)
        assert plan.rows(s)[j] == y
    if len(set(runs)) == 1:  # equal runs are round-robin bands
        assert [plan.count(s) for s in range(n)] == [rm.shard_rows(H_, runs[0], n, s) for s in range(n)]


def test_cycle_rows_rejects_bad_parts():
    for args in ((10, 0, 0, 1), (10, 4, 3, 2), (10, 4, -1, 2), (10, 4, 0, 0), (0, 4, 0, 1)):
        with pytest.raises(rm.RmError):
            rm.cycle_rows(*args)


@pytest.mark.parametrize("H_,band,n", [(37, 16, 2), (4096, 16, 8), (1080, 27, 8), (9, 4, 5)])
def test_shard_plan_matches_c_abi(H_, band, n):
    plan = ShardPlan(8, H_, band, n)
    for s in range(n):
        assert plan.count(s) == rm.shard_rows(H_, band, n, s) == len(plan.rows(s))
    idx = plan.gathered_index()
    assert len(set(idx)) == H_
    for y in range(0, H_, max(1, H_ // 50)):
        s, j = plan.slot_of_row(y)
        assert plan.rows(s)[j] == y
