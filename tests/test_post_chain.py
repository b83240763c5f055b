"""The reference's post passes of a frame, chained as main.cpp:209-214 runs
them (rm_post_chain): FXAA (post.frag:16-61) into postTexture, its mip chain
(generateMipmap), bloom.frag:14-43 of it.

* bit for bit the oracle's chain, oracle.bloom(oracle.fxaa(frame)), on frames
  whose mips take the exact-halving pyramid (256 x 2560, 512 x 512) and the
  per-level resample (200 x 150);
* bit for bit rm_fxaa followed by rm_bloom, up to the C3 frame (4096^2);
* bench.post_plan's restatement of the C++ bloom_plan's mip path.
"""
import numpy as np
import pytest

import oracle

# (W, H, pyramid): the exact-halving pyramid needs W, H multiples of 2^d2
# (d2 = floor(log2(0.05 H)) + 1) and 5 to 8 levels below its start
SIZES = [(256, 2560, True), (4096, 4096, True), (512, 512, True), (1920, 1080, False), (200, 150, False),
         (8192, 8192, True)]


@pytest.mark.parametrize("W,H,pyramid", SIZES)
def test_mip_path(W, H, pyramid):
    import bench
    assert bench.post_plan(W, H)["pyramid"] == pyramid


def _frame(R, W, H, kind):
    import raymarching_amd as rm
    import torch
    if kind == "random":
        g = torch.Generator(device="cuda").manual_seed(W * 7 + H)
        return torch.randint(-2**31, 2**31 - 1, (H, W), dtype=torch.int32, device="cuda", generator=g)
    R.load_scene(rm.SCENE_FILES["T"])
    p = rm.POSES["P1"]
    R.set_pose(p["pos"], p["mouse"], p["time"])
    R.set_params(max_steps=128, count_evals=0)
    return R.render_rgba8(W, H)


@pytest.fixture(scope="module")
def R(torch_cuda):
    import raymarching_amd as rm
    r = rm.Renderer(0)
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(256, 2560), (200, 150), (512, 512)])
@pytest.mark.parametrize("kind", ["render", "random"])
def test_post_chain_bit_exact_vs_oracle_chain(R, W, H, kind):
    f8 = _frame(R, W, H, kind)
    mid, out = R.post_chain(f8)
    src = f8.cpu().numpy().view(np.uint32)
    ref_mid, _ = oracle.fxaa(src)
    ref_out, _ = oracle.bloom(ref_mid)
    assert np.array_equal(mid.cpu().numpy().view(np.uint32), ref_mid)
    got = out.cpu().numpy().view(np.uint32)
    nd = int((got != ref_out).sum())
    assert nd == 0, f"{nd} pixels of the chained frame differ from the oracle's chain"


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(4096, 4096), (1920, 1080), (256, 2560)])
def test_post_chain_equals_fxaa_then_bloom(R, W, H):
    import torch
    f8 = _frame(R, W, H, "render")
    mid, out = R.post_chain(f8)
    m2 = R.fxaa(f8)
    o2 = R.bloom(m2)
    torch.cuda.synchronize()
    assert torch.equal(mid, m2)
    assert torch.equal(out, o2)
    # a second chain on the same context (cached run tables) gives the same frame
    mid3, out3 = R.post_chain(f8)
    assert torch.equal(out3, o2)


@pytest.mark.gpu
def test_post_chain_rejects_aliasing(R):
    import torch
    import raymarching_amd as rm
    f8 = torch.zeros((64, 64), dtype=torch.int32, device="cuda")
    with pytest.raises(rm.RmError):
        R.post_chain(f8, mid=f8)
