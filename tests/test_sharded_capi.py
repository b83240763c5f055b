"""rm_render_sharded (librm.so's RCCL path, include/rm.h "Multi-GPU").

CPU: the layout the C ABI reports (rm_sharded_layout) against ShardPlan, and a
two-rank gloo run of the host-side plan -- each rank's RGB8 wire built from
the oracle's rows at the offsets the C layout gives, gathered to rank 0 and
de-interleaved there -- against a one-process frame.  GPU: one-rank
communicators (rm_comm_init_rank, rm_comm_init_all) through the C ABI, bit for
bit against rm_render_rgba8.  N > 1 over RCCL runs only on a multi-GPU node
(the driver's scaling run): RCCL refuses two ranks on one GPU."""
import os
import socket

import numpy as np
import pytest

import raymarching_amd as rm
from raymarching_amd.frame import ShardPlan

POSE = rm.POSES["P3"]


@pytest.mark.parametrize("W,H,band,n", [(4096, 4096, 16, 8), (1920, 1080, 27, 8), (61, 50, 7, 3), (8, 5, 16, 4),
                                        (33, 17, 1, 17)])
def test_sharded_layout_matches_shard_plan(W, H, band, n):
    plan = ShardPlan(W, H, band, n)
    for r in range(n):
        L = rm.sharded_layout(W, H, band, n, r)
        assert L["rows_mine"] == plan.count(r)
        assert L["rows_per_shard"] == plan.rows_per_shard
        assert L["wire_bytes"] == plan.rows_per_shard * 3 * W
        assert L["gathered_bytes"] == n * L["wire_bytes"]


def test_sharded_layout_rejects_bad_arguments():
    for args in ((0, 8, 16, 2, 0), (8, 8, 0, 2, 0), (8, 8, 16, 2, 2), (8, 8, 16, 0, 0)):
        with pytest.raises(rm.RmError):
            rm.sharded_layout(*args)


def unorm8_words(rgba):
    q = np.clip(np.rint(np.clip(np.nan_to_num(rgba, nan=0.0), 0, 1) * 255.0), 0, 255).astype(np.uint32)
    return q[..., 0] | (q[..., 1] << 8) | (q[..., 2] << 16) | (q[..., 3] << 24)


def _plan_worker(rank, world, port, W, H, band, q):
    import torch
    import torch.distributed as dist

    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = rm.sharded_layout(W, H, band, world, rank)
    rows = [y for y in range(H) if (y // band) % world == rank]
    assert len(rows) == L["rows_mine"]
    wire = np.zeros(L["wire_bytes"], np.uint8)  # rows past rows_mine: padding
    if rows:
        img, _ = oracle.render_rows("T", W, H, rows, pos=POSE["pos"], mouse=POSE["mouse"], time=POSE["time"])
        rgb = unorm8_words(img).view(np.uint8).reshape(len(rows), W, 4)[..., :3]  # rm_pack_rgb8
        wire[: len(rows) * 3 * W] = rgb.reshape(-1)
    t = torch.from_numpy(wire)
    got = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=got, dst=0)
    if rank == 0:
        gathered = torch.cat(got).numpy()
        assert gathered.size == L["gathered_bytes"]
        frame = np.zeros((H, W), np.uint32)
        for y in range(H):  # rm_deinterleave_rgb8: rank r's wire at r * wire_bytes
            gb, rr = divmod(y, band)
            r, j = gb % world, (gb // world) * band + rr
            off = r * L["wire_bytes"] + j * 3 * W
            px = gathered[off: off + 3 * W].reshape(W, 3).astype(np.uint32)
            frame[y] = px[:, 0] | (px[:, 1] << 8) | (px[:, 2] << 16) | (255 << 24)
        q.put(frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 4), (3, 1)])
def test_two_rank_host_plan_reassembles_the_frame(world, band):
    import torch.multiprocessing as mp

    import oracle
    W, H = 24, 19
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, W, H, band, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = oracle.render("T", W, H, pos=POSE["pos"], mouse=POSE["mouse"], time=POSE["time"])
    np.testing.assert_array_equal(frame, unorm8_words(full))


# ------------------------------------------------------------------ GPU


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,band", [(96, 64, 16), (77, 45, 4), (256, 256, 16)])
def test_one_rank_communicator_equals_render_rgba8(torch_cuda, W, H, band):
    torch = torch_cuda
    r = rm.Renderer(0)
    r.load_scene("template.frag")
    r.set_pose(POSE["pos"], POSE["mouse"], POSE["time"])
    r.set_params(max_steps=128, count_evals=0)
    ref = r.render_rgba8(W, H)
    c = rm.Comm(r, 1, 0, rm.comm_get_id())
    assert c.uses_rccl  # ncclCommInitRank + ncclGather over a one-rank communicator
    frame, st = c.render(W, H, band, stats=True)
    assert torch.equal(frame, ref)
    assert st["pixels"] == W * H and st["kernel_ms"] > 0
    (c1,) = rm.Comm.init_all([r])
    assert c1.uses_rccl  # ncclCommInitAll
    f1 = rm.Comm.render_all([c1], W, H, band)
    torch.cuda.synchronize()
    assert torch.equal(f1, ref)
    c.close()
    c1.close()
    r.close()


@pytest.mark.gpu
def test_comm_unique_id_and_errors(torch_cuda):
    cid = rm.comm_get_id()  # loads RCCL (ncclGetUniqueId)
    assert len(cid) == 128 and any(cid)
    r = rm.Renderer(0)
    r.load_scene("template.frag")
    c = rm.Comm(r, 1, 0, cid)
    with pytest.raises(rm.RmError):
        c.render(0, 8, 4)
    assert rm.lib().rm_render_sharded(c._h, 8, 8, 4, None, None) == 1  # rank 0 needs a frame
    c.close()
    r.close()
