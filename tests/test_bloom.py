"""The bloom post pass: shaders/post/bloom.frag:14-43
over the mip chain main.cpp:212-214 builds (setSmooth + generateMipmap).

Pinning: tests/golden/BLOOM_*.npz hold SwiftShader's glGenerateMipmap levels
and bloom.frag output for two FXAA outputs of ray-march goldens and three
synthetic images (power-of-two and odd sizes).  The oracle's mip levels match
SwiftShader bit for bit on even sizes; on odd sizes (a bilinear resample at
non-half-texel positions) within 1 LSB on <= 5 % of the texels.  SwiftShader filters unorm8 texels in
fixed point, the oracle and the HIP path in float32, so the bloom output is
within 1 LSB everywhere and identical on >= 90 % of the pixels (the LSB
itself is unpinned).  The HIP path (rm_bloom) is bit-exact against the
oracle: same float operations in the same order, no contraction.
"""
import glob
import json
import os

import numpy as np
import pytest

import oracle
import raymarching_amd as rm

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "BLOOM_*.npz")))
IDS = [os.path.basename(p)[:-4] for p in GOLDEN]


def channels(a):
    a = np.asarray(a, np.uint32)
    return np.stack([(a >> (8 * c)) & 255 for c in range(4)], -1).astype(np.int64)


def test_goldens_present():
    assert len(GOLDEN) >= 5


@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_oracle_mips_match_swiftshader(path):
    z = np.load(path, allow_pickle=False)
    m = json.loads(str(z["meta"]))
    cur = z["input"]
    k = 1
    while f"mip{k}" in z:
        ref = z[f"mip{k}"]
        got = oracle.mip_down(cur)
        assert got.shape == ref.shape
        d = np.abs(channels(got) - channels(ref))
        even = cur.shape[0] % 2 == 0 and cur.shape[1] % 2 == 0 or min(cur.shape) == 1
        if even:
            assert d.max() == 0, (k, float(np.mean(d.max(-1) > 0)))
        else:
            assert d.max() <= 1 and np.mean(d.max(-1) == 0) >= 0.95, (k, m["W"], m["H"])
        cur = ref  # continue from SwiftShader's level
        k += 1


@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_oracle_bloom_matches_swiftshader(path):
    z = np.load(path, allow_pickle=False)
    out, _ = oracle.bloom(z["input"])
    d = np.abs(channels(out) - channels(z["output"]))
    assert d.max() <= 1
    assert np.mean(d.max(-1) == 0) >= 0.90


@pytest.mark.parametrize("W,H,d1,d2", [(64, 64, 1, 2), (1920, 1080, 5, 6), (4096, 4096, 7, 8), (19, 19, 0, 0),
                                       (8, 1024, 5, 6), (4096, 16, 0, 0)])
def test_lod_levels(W, H, d1, d2):
    lod, a, b = oracle.bloom_levels(W, H)
    assert np.isclose(lod, np.log2(0.05 * H), atol=1e-5)
    assert (a, b) == (d1, d2)


def _per_tap_bloom(img, levels):
    """bloom.frag for lod > 0 by its definition, in float64: 25 bilinear taps
    per level (CLAMP_TO_EDGE, texel centres), the two levels blended by fr."""
    H, W = img.shape
    lod, d1, d2 = oracle.bloom_levels(W, H)
    fr = lod - np.floor(lod)
    G = np.array([[41, 26, 7], [26, 16, 4], [7, 4, 1]]) / 273.0
    u = (np.arange(W) + 0.5) / W
    v = 1.0 - (np.arange(H) + 0.5) / H
    c = channels(img)[..., :3] / 255.0

    def bilinear(L, uu, vv):
        h, w = L.shape[:2]
        x = uu * w - 0.5
        y = vv * h - 0.5
        fx, fy = np.floor(x), np.floor(y)
        a, b = (x - fx)[None, :, None], (y - fy)[:, None, None]
        x0, x1 = np.clip(fx, 0, w - 1).astype(int), np.clip(fx + 1, 0, w - 1).astype(int)
        y0, y1 = np.clip(fy, 0, h - 1).astype(int), np.clip(fy + 1, 0, h - 1).astype(int)
        return ((1 - b) * ((1 - a) * L[np.ix_(y0, x0)] + a * L[np.ix_(y0, x1)])
                + b * ((1 - a) * L[np.ix_(y1, x0)] + a * L[np.ix_(y1, x1)]))

    lv = [c] + [channels(m)[..., :3] / 255.0 for m in levels]  # lv[k]: level k
    acc = 0.0
    for L, wgt in ((lv[d1], 1 - fr), (lv[d2], fr)):
        for j in range(-2, 3):
            for i in range(-2, 3):
                acc = acc + wgt * G[abs(i), abs(j)] * bilinear(L, u + i * (H / W) * 0.05, v + j * 0.05)
    base = bilinear(c, u, v)
    out = np.clip(base + np.maximum(acc - 0.3, 0.0), 0.0, 1.0)
    return np.rint(out * 255.0).astype(np.int64)


@pytest.mark.parametrize("W,H", [(256, 256), (300, 200), (96, 54), (64, 700), (300, 30), (1000, 24)])
def test_oracle_runs_equal_per_tap_sum(W, H):
    """The oracle (and the HIP path, bit-exact to it) sums each level's 25 taps
    as one bilinear polynomial per (column run, row run) pair of cells; that is
    the per-tap sum of bloom.frag rounded differently: within 1 LSB of a
    float64 per-tap evaluation over the oracle's own mip levels, and identical
    on >= 99.5 % of the channels."""
    rng = np.random.default_rng(W * 31 + H)
    img = rng.integers(0, 2 ** 32, (H, W), dtype=np.uint64).astype(np.uint32)
    out, levels = oracle.bloom(img)
    ref = _per_tap_bloom(img, levels)
    d = np.abs(channels(out)[..., :3] - ref)
    assert d.max() <= 1
    assert np.mean(d == 0) >= 0.995, float(np.mean(d == 0))


# ------------------------------------------------------------ GPU


@pytest.fixture(scope="module")
def R(torch_cuda):
    r = rm.Renderer(0)
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_hip_bloom_bit_exact_vs_oracle(R, path):
    import torch
    z = np.load(path, allow_pickle=False)
    img = torch.from_numpy(z["input"].astype(np.int32)).cuda()
    out = R.bloom(img).cpu().numpy().astype(np.uint32)
    ref, _ = oracle.bloom(z["input"])
    assert np.array_equal(out, ref), float(np.mean(out != ref))
    d = np.abs(channels(out) - channels(z["output"]))
    assert d.max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(1, 1), (7, 3), (33, 65), (1920, 1080), (4096, 16), (16, 4096), (300, 2000),
                                 (2048, 1152), (4096, 2048), (4096, 4096),  # (pyramid kernels <1>, <2>, <3>)
                                 (300, 30), (16384, 24)])  # (0 < lod < 1: level d1 is the frame itself)
def test_hip_bloom_ragged_sizes(R, W, H):
    import torch
    rng = np.random.default_rng(W * 7919 + H)
    src = rng.integers(0, 2 ** 32, (H, W), dtype=np.uint64).astype(np.uint32)
    out = R.bloom(torch.from_numpy(src.astype(np.int32)).cuda()).cpu().numpy().astype(np.uint32)
    ref, _ = oracle.bloom(src)
    assert np.array_equal(out, ref), float(np.mean(out != ref))


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(1024, 512), (1000, 600)])  # exact-halving pyramid / per-level mip launches
def test_hip_bloom_cached_run_tables(R, W, H):
    """The run tables depend on W x H only and are kept between calls of one
    size on one stream: a second image of the same size reuses them, a change
    of size or of the context's stream rebuilds them -- bit-exact every time."""
    import torch
    rng = np.random.default_rng(W + 7 * H)
    imgs = [rng.integers(0, 2 ** 32, (H, W), dtype=np.uint64).astype(np.uint32) for _ in range(2)]
    small = rng.integers(0, 2 ** 32, (H // 2, W // 2), dtype=np.uint64).astype(np.uint32)

    def run(img):
        out = R.bloom(torch.from_numpy(img.astype(np.int32)).cuda())
        torch.cuda.synchronize()
        return out.cpu().numpy().astype(np.uint32)

    for img in (imgs[0], imgs[1], small, imgs[1]):  # cached, cached, rebuilt (size), rebuilt (size)
        assert np.array_equal(run(img), oracle.bloom(img)[0])
    s = torch.cuda.Stream()
    try:
        with torch.cuda.stream(s):
            R.set_stream(s)
            got = run(imgs[0])  # rebuilt (stream)
    finally:
        R.set_stream(torch.cuda.current_stream())
    assert np.array_equal(got, oracle.bloom(imgs[0])[0])
    assert np.array_equal(run(imgs[1]), oracle.bloom(imgs[1])[0])


@pytest.mark.gpu
def test_hip_bloom_of_a_rendered_frame(R):
    """The reference's order: ray-march pass -> FXAA -> bloom, all on the GPU."""
    import torch
    R.load_scene("template.frag")
    R.set_pose(*[rm.POSES["P0"][k] for k in ("pos", "mouse", "time")])
    R.set_params(max_steps=128, count_evals=0)
    frame = R.render_rgba8(512, 288)
    aa = R.fxaa(frame)
    out = R.bloom(aa).cpu().numpy().astype(np.uint32)
    ref, _ = oracle.bloom(aa.cpu().numpy().astype(np.uint32))
    assert np.array_equal(out, ref)
    assert torch.cuda.is_available()
