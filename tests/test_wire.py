"""The compressed wire of RGBA8 row parts (raymarching_amd/csrc/rm_wire_tile.h,
rm_wire.hip): the numpy restatement (tests/wire_codec.py)
round-trips on CPU; on the GPU both encoders -- the rows encoder and the
render kernel's epilogue (rm_render_cycle_rows_wire) -- write the
restatement's bytes exactly and the decoder rebuilds every part's frame rows
bit for bit."""
import numpy as np
import pytest

import raymarching_amd as rm
from tests import wire_codec


@pytest.fixture(scope="module")
def R(torch_cuda):
    r = rm.Renderer(0)
    yield r
    r.close()


def _smooth(n, W, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:n, 0:W]
    r = (x * 255 // max(W - 1, 1)).astype(np.uint32)
    g = ((y * 7 + x // 9) % 256).astype(np.uint32)
    b = np.where(rng.random((n, W)) < 0.02, rng.integers(0, 256, (n, W)), 128).astype(np.uint32)
    return r | (g << 8) | (b << 16) | np.uint32(0xFF000000)


def _noise(n, W, seed=1):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2**24, (n, W), dtype=np.uint32) | np.uint32(0xFF000000)


@pytest.mark.parametrize("n,W", [(3, 64), (5, 97), (2, 200), (1, 1), (16, 4096), (9, 17)])
@pytest.mark.parametrize("kind", ["smooth", "noise", "flat"])
def test_numpy_codec_round_trip(n, W, kind):
    img = {"smooth": _smooth, "noise": _noise}.get(kind, lambda n, W: np.full((n, W), 0xFF102030, np.uint32))(n, W)
    msg = wire_codec.encode(img)
    assert int(np.frombuffer(msg[:8].tobytes(), np.int64)[0]) == msg.size
    assert msg.size <= rm.wire_capacity(W, n)
    assert np.array_equal(wire_codec.decode(msg, n, W), img)
    T = ((W + 7) // 8) * ((n + 7) // 8)
    if kind == "flat" and W % 8 == 0 and n % 8 == 0:  # one header word per tile plus the offset table
        assert msg.size == wire_codec.header_bytes(T) + 8 * T


def test_tile_code_differences_run_along_rows_and_the_first_column():
    """A tile whose rows are ramps and whose first column is another ramp needs
    one bit plane per channel that changes by one: differences are taken to
    the left, and to the pixel above only in the first column."""
    y, x = np.mgrid[0:8, 0:8]
    r = (10 + x + 3 * y).astype(np.uint32)  # +1 along rows, +3 down the first column
    p = (r | (np.uint32(50) << 8) | (np.uint32(7) << 16) | np.uint32(0xFF000000)).ravel()
    w = wire_codec.tile_words(p)
    assert (w[0] >> 24) & 15 == 3 and (w[0] >> 28) & 15 == 0 and (w[0] >> 32) & 15 == 0  # zigzag(3) = 6: 3 bits
    assert w[0] & 0xFFFFFF == 10 | (50 << 8) | (7 << 16)


def test_capacity_and_workspace_sizes():
    T = 512 * 4096 // 64
    assert rm.wire_capacity(4096, 512) == wire_codec.header_bytes(T) + 8 * 25 * T
    # word-major slots, a count byte per tile, a base per 64-tile chunk
    assert rm.wire_workspace_bytes(4096, 512) == ((8 * 25 * T + T + 3) & ~3) + 4 * ((T + 63) // 64)
    with pytest.raises(ValueError):
        rm.wire_capacity(0, 4)


def _gpu_encode(R, torch, img):
    n, W = img.shape
    rows = torch.from_numpy(img.view(np.int32)).cuda()
    msg = torch.zeros(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda")
    ws = torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda")
    size = torch.zeros(1, dtype=torch.int64, device="cuda")
    R.wire_encode(rows, msg, ws, size)
    torch.cuda.synchronize()
    return msg, int(size.item())


@pytest.mark.gpu
@pytest.mark.parametrize("n,W", [(3, 64), (5, 97), (2, 200), (7, 4096)])
@pytest.mark.parametrize("kind", ["smooth", "noise"])
def test_gpu_encoder_writes_the_restated_bytes(R, torch_cuda, n, W, kind):
    torch = torch_cuda
    img = (_smooth if kind == "smooth" else _noise)(n, W)
    ref = wire_codec.encode(img)
    msg, size = _gpu_encode(R, torch, img)
    assert size == ref.size
    assert np.array_equal(msg[:size].cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,runs", [(96, 70, (13, 8)), (97, 61, (1, 5, 2)), (4096, 512, (16, 16, 16, 16))])
def test_gpu_wire_rebuilds_rendered_parts(R, torch_cuda, W, H, runs):
    """A rendered frame's parts: rank 0's rows scattered, every other part
    encoded on the GPU and decoded into the frame: equal to rm_render_rgba8."""
    torch = torch_cuda
    from raymarching_amd.frame import ShardPlan
    R.load_scene(rm.SCENE_FILES["T"])
    R.set_uniform("u_resolution", W, H)
    p = rm.POSES["P1"]
    R.set_pose(p["pos"], p["mouse"], p["time"])
    R.set_params(max_steps=128, count_evals=0)
    ref = R.render_rgba8(W, H)
    plan = ShardPlan(W, H, runs[-1], len(runs), runs)
    frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    sizes = []
    for s in range(len(runs)):
        n = plan.count(s)
        loc = torch.empty((n, W), dtype=torch.int32, device="cuda")
        R.render_cycle_rows(W, H, plan.cycle, plan.offsets[s], runs[s], 0, n, loc)
        if s == 0:
            R.scatter_part_rgba8(W, H, plan.cycle, plan.offsets[s], runs[s], n, loc, frame)
            continue
        msg = torch.empty(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda")
        ws = torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda")
        size = torch.zeros(1, dtype=torch.int64, device="cuda")
        R.wire_encode(loc, msg, ws, size)
        # the message as it would arrive: only its `size` bytes
        got = torch.zeros_like(msg)
        torch.cuda.synchronize()
        k = int(size.item())
        got[:k] = msg[:k]
        R.wire_decode(W, H, plan.cycle, plan.offsets[s], runs[s], n, got, frame)
        sizes.append((k, n * W * 3))
    torch.cuda.synchronize()
    assert torch.equal(frame, ref)
    if W == 4096:  # a rendered frame compresses
        assert all(k * 2 < raw for k, raw in sizes), sizes


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["T", "O"])
@pytest.mark.parametrize("W,H,runs", [(96, 70, (13, 8)), (97, 61, (1, 5, 2)), (4096, 512, (16, 16, 16, 16))])
def test_gpu_render_epilogue_writes_the_encoders_message(R, torch_cuda, scene, W, H, runs):
    """rm_render_cycle_rows_wire: the render kernel encodes its own tiles, and
    the message is byte for byte the rows encoder's (and the numpy
    restatement's) of the rows rm_render_cycle_rows_rgba8 renders; it decodes
    to them (adaptive dispatch order on, so the tiles run out of order)."""
    torch = torch_cuda
    from raymarching_amd.frame import ShardPlan
    R.load_scene(rm.SCENE_FILES[scene])
    R.set_uniform("u_resolution", W, H)
    p = rm.POSES["P1"]
    R.set_pose(p["pos"], p["mouse"], p["time"])
    R.set_params(max_steps=128 if scene == "T" else 256, count_evals=0, schedule=1)
    plan = ShardPlan(W, H, runs[-1], len(runs), runs)
    for s in range(1, len(runs)):
        n = plan.count(s)
        loc = torch.empty((n, W), dtype=torch.int32, device="cuda")
        msg = torch.zeros(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda")
        ws = torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda")
        size = torch.zeros(1, dtype=torch.int64, device="cuda")
        for _ in range(3):  # (the second and third launch dispatch costliest tiles first)
            R.render_cycle_rows(W, H, plan.cycle, plan.offsets[s], runs[s], 0, n, loc)
            R.render_cycle_rows_wire(W, H, plan.cycle, plan.offsets[s], runs[s], 0, n, msg, ws, size)
        torch.cuda.synchronize()
        k = int(size.item())
        ref_gpu, k2 = _gpu_encode(R, torch, loc.cpu().numpy().view(np.uint32))
        assert k == k2
        assert torch.equal(msg[:k], ref_gpu[:k])
        if n * W <= 97 * 61:
            assert np.array_equal(msg[:k].cpu().numpy(), wire_codec.encode(loc.cpu().numpy().view(np.uint32)))
        frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        R.wire_decode(W, H, plan.cycle, plan.offsets[s], runs[s], n, msg, frame)
        R.scatter_part_rgba8(W, H, plan.cycle, plan.offsets[s], runs[s], n, loc, frame2 := torch.zeros_like(frame))
        torch.cuda.synchronize()
        assert torch.equal(frame, frame2)


@pytest.mark.gpu
def test_gpu_render_wire_empty_part(R, torch_cuda):
    torch = torch_cuda
    R.load_scene(rm.SCENE_FILES["T"])
    msg = torch.full((rm.wire_capacity(64, 0),), 7, dtype=torch.uint8, device="cuda")
    ws = torch.empty(max(1, rm.wire_workspace_bytes(64, 0)), dtype=torch.uint8, device="cuda")
    size = torch.zeros(1, dtype=torch.int64, device="cuda")
    R.render_cycle_rows_wire(64, 8, 16, 8, 8, 0, 0, msg, ws, size)  # H = 8 rows, the part (8, 8) holds none
    torch.cuda.synchronize()
    assert int(size.item()) == 8


@pytest.mark.gpu
def test_gpu_wire_rejects_bad_parts(R, torch_cuda):
    torch = torch_cuda
    frame = torch.zeros((8, 64), dtype=torch.int32, device="cuda")
    msg = torch.zeros(rm.wire_capacity(64, 8), dtype=torch.uint8, device="cuda")
    with pytest.raises(rm.RmError):
        R.wire_decode(64, 8, 4, 3, 2, 1, msg, frame)  # offset + run > cycle
    with pytest.raises(rm.RmError):
        R.wire_decode(64, 8, 4, 0, 2, 5, msg, frame)  # more rows than the part has


def test_delta_frame_size_check_on_every_rank():
    """DeltaFrame._check_sizes needs only the plan (no receive buffers), so
    every rank runs it on the gathered sizes before any send or receive: a
    rank reporting more than its part's wire capacity fails them all."""
    from types import SimpleNamespace

    from raymarching_amd.frame import DeltaFrame, ShardPlan
    plan = ShardPlan(4096, 4096, 16, 3)
    stub = SimpleNamespace(world=3, plan=plan)
    caps = [rm.wire_capacity(4096, plan.count(q)) for q in range(3)]
    DeltaFrame._check_sizes(stub, [0, caps[1], 17])
    with pytest.raises(RuntimeError, match="rank 2"):
        DeltaFrame._check_sizes(stub, [0, 5, caps[2] + 1])
    with pytest.raises(RuntimeError, match="rank 1"):
        DeltaFrame._check_sizes(stub, [0, -1, 5])
