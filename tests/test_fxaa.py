"""FXAA post pass (post.frag:16-61, :135-144): the oracle against SwiftShader
renders of post.frag (tests/golden/FXAA_*.npz), and the HIP kernel against the
oracle (bit for bit) and the goldens."""
import glob
import os

import numpy as np
import pytest

import oracle

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "FXAA_*.npz")))


def bytes_of(u32):
    return np.ascontiguousarray(u32, np.uint32).view(np.uint8).reshape(u32.shape + (4,)).astype(np.int64)


def lsb_stats(a, b):
    d = np.abs(bytes_of(a) - bytes_of(b)).max(-1)
    return float(np.mean(d == 0)), float(np.mean(d <= 1)), int(d.max())


def test_fxaa_goldens_present():
    assert len(GOLD) == 3


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_oracle_fxaa_matches_reference_glsl(path):
    z = np.load(path, allow_pickle=False)
    out, _ = oracle.fxaa(z["input"])
    exact, within1, mx = lsb_stats(out, z["output"])
    # SwiftShader's float->unorm8 store and texel fetch round slightly differently
    assert within1 >= 0.999 and exact >= 0.85, (exact, within1, mx)


def test_fxaa_flat_and_flip():
    img = np.full((20, 30), 0xFF336699, np.uint32)
    out, _ = oracle.fxaa(img)
    assert np.array_equal(out, img)
    # a horizontal gradient without edges comes back flipped vertically
    g = (np.arange(20)[:, None] * 3 + 0xFF000000 + np.zeros((1, 30), np.int64)).astype(np.uint32)
    out, _ = oracle.fxaa(g)
    assert np.array_equal(out, g[::-1])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_hip_fxaa_bit_exact_vs_oracle(path, torch_cuda):
    import raymarching_amd as rm
    torch = torch_cuda
    z = np.load(path, allow_pickle=False)
    r = rm.Renderer(0)
    inp = torch.from_numpy(z["input"].view(np.int32)).cuda()
    out = r.fxaa(inp).cpu().numpy().view(np.uint32)
    ref, _ = oracle.fxaa(z["input"])
    assert np.array_equal(out, ref)
    exact, within1, _ = lsb_stats(out, z["output"])
    assert within1 >= 0.999 and exact >= 0.85
    r.close()


@pytest.mark.gpu
def test_hip_fxaa_full_frame(torch_cuda):
    """FXAA of a 4096^2 scene-T frame (the hot path's RGBA8 output) equals the
    oracle's FXAA of the same bytes."""
    import raymarching_amd as rm
    r = rm.Renderer(0)
    r.load_scene("template.frag")
    p = rm.POSES["P0"]
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=256)
    f8 = r.render_rgba8(4096, 4096)
    out = r.fxaa(f8).cpu().numpy().view(np.uint32)
    ref, _ = oracle.fxaa(f8.cpu().numpy().view(np.uint32))
    assert np.array_equal(out, ref)
    r.close()
