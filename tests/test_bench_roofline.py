"""bench.py's roofline(): frac comes from PMC-counted FP32 FLOP only -- for the
counted launch itself, or per executed ray-step for a share of it (N > 1) --
never from the instrumented tally, and no rate in it exceeds its peak (host
logic, no GPU)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

PMC = json.load(open(os.path.join(ROOT, "profiles", "pmc_counters.json")))
C3 = PMC["T_4096x4096_256_P0"]


def _rates(d, path=""):
    """(path, value, peak) of every achieved/peak pair in the line."""
    out = []
    if isinstance(d, dict):
        if d.get("achieved") is not None and d.get("peak"):
            out.append((path, d["achieved"], d["peak"]))
        for k, v in d.items():
            out += _rates(v, f"{path}.{k}")
    return out


def test_exact_launch_uses_counted_flop():
    ms = C3["avg_kernel_ns_trace"] / 1e6
    r = bench.roofline(C3, ms, C3["executed_ray_steps_per_launch"], 4096 * 4096 * 4, 9e13, 1e9)
    flop = bench.pmc_flop(C3)[0]
    assert r["flop_per_launch"] == pytest.approx(flop)
    assert r["frac"] == pytest.approx(flop / (ms / 1e3) / 1e12 / bench.PEAK_FP32_TFLOPS)
    assert 0.2 < r["frac"] < 0.5
    # the tally (here a nonsense 9e13) stays out of frac
    assert r["tally_frac"] > 1 and r["frac"] < 1
    assert r["hbm"]["counter_gbs"] == pytest.approx(C3["hbm_bytes_per_launch"] / (ms / 1e3) / 1e9)
    assert "reference_equivalent_tflops" not in r and "tally_tflops" not in r
    assert all(v <= p for _, v, p in _rates(r))


@pytest.mark.parametrize("share", [0.5, 0.8, 0.125])
def test_rank_share_priced_per_executed_step(share):
    """A rank that executes a share of the frame's steps in the same time per
    step as the whole frame gets the N = 1 fraction, whatever its share."""
    ms = C3["avg_kernel_ns_trace"] / 1e6
    base = bench.roofline(C3, ms, C3["executed_ray_steps_per_launch"], 1, None, None)
    steps = int(C3["executed_ray_steps_per_launch"] * share)
    r = bench.roofline(C3, ms * share, steps, 1, 5e10, 1e9, exact=False, rows_frac=share)
    assert r["frac"] == pytest.approx(base["frac"], rel=1e-6)
    assert r["traffic"] == pytest.approx(C3["hbm_bytes_per_launch"] * share)
    assert "per executed ray-step" in r["flop_source"]
    assert "valu_issue" not in r  # issue fractions are counters of the counted launch only


def test_tally_never_becomes_frac():
    """No counters (or counters without the executed-steps anchor for a share):
    frac is null with a reason, whatever the tally says."""
    r = bench.roofline({}, 0.45, 5e8, 1, 5.3e10, 1e9)
    assert r["frac"] is None and r["achieved"] is None and "no PMC" in r["frac_null_reason"]
    assert r["tally_frac"] == pytest.approx(5.3e10 / 0.45e-3 / 1e12 / bench.PEAK_FP32_TFLOPS)
    no_anchor = {k: v for k, v in C3.items() if k != "executed_ray_steps_per_launch"}
    r = bench.roofline(no_anchor, 0.2, 2.6e8, 1, 5.3e10, 1e9, exact=False, rows_frac=0.5)
    assert r["frac"] is None and "executed_ray_steps" in r["frac_null_reason"]


def test_no_rows_no_launch():
    r = bench.roofline(C3, 0.0, 0, 0, None, None, exact=False)
    assert r["frac"] is None


def test_r04_n2_rehearsal_tally_is_not_the_roofline():
    """Round 4's gloo N = 2 rehearsal line (balanced runs [1089, 16]: rank 0
    rendered 98.6 % of the rows in 0.4535 ms) printed frac 0.742 from the
    tally.  Priced per executed ray-step it is an N = 1-like fraction (the
    counters are round 5's, whose kernel does fewer FLOP per ray-step than
    round 4's, so only the order of magnitude is compared here)."""
    n2 = json.load(open(os.path.join(ROOT, "profiles", "r04", "bench_n2_gloo_r04final2.json")))
    runs = n2["balance"]["runs"]
    share = runs[0] / sum(runs)
    steps = int(C3["executed_ray_steps_per_launch"] * share)
    r = bench.roofline(C3, n2["kernel_ms_per_rank"][0], steps, 1, n2["roofline"]["tally_flop_per_launch"], None,
                       exact=False, rows_frac=share)
    assert n2["roofline"]["frac"] > 0.7  # the old, tally-based figure
    assert 0.25 < r["frac"] < 0.45
    assert r["tally_frac"] > 0.7


def test_r05_n2_rehearsal_within_5pct_of_n1():
    """Round 5's gloo N = 2 rehearsal and the N = 1 C3 line of the same
    validation run (same build, profiles/r05/*_r05k.json, the final pass): rank 0's share,
    priced per executed ray-step, lands within 5 % of the N = 1 counted
    fraction, as the same kernel over nearly the same rows must; the tally
    stays in tally_frac."""
    lines = open(os.path.join(ROOT, "profiles", "r05", "bench_n2_gloo_r05k.json")).read().splitlines()
    n2 = json.loads([ln for ln in lines if ln.startswith("{")][-1])  # (gloo's connection log precedes the line)
    n1 = json.load(open(os.path.join(ROOT, "profiles", "r05", "bench_C3_r05k.json")))
    assert n2["n_gpus"] == 2 and n1["n_gpus"] == 1
    f1, f2 = n1["roofline"]["frac"], n2["roofline"]["frac"]
    assert f2 == pytest.approx(f1, rel=0.05)
    assert "per executed ray-step" in n2["roofline"]["flop_source"]
    assert n2["roofline"]["tally_frac"] > 0.7 > f2
    assert all(v <= p for _, v, p in _rates(n2))


@pytest.mark.parametrize("scale", [0.8, 1.25])
def test_stale_counters_give_no_frac(scale):
    """Counters whose launch took > 10 % longer or shorter than the measured one
    are another build's: frac, traffic and the issue fractions are null, with
    the reason (round 5: a C5 line priced with the previous build's counters
    showed a VALU issue fraction above 1)."""
    ms = C3["avg_kernel_ns_trace"] / 1e6 * scale
    r = bench.roofline(C3, ms, C3["executed_ray_steps_per_launch"], 4096 * 4096 * 4, 5e10, 1e9)
    assert r["frac"] is None and r["traffic"] is None
    assert "stale" in r["frac_null_reason"]
    assert "valu_issue" not in r and "salu_issue" not in r
    ok = bench.roofline(C3, C3["avg_kernel_ns_trace"] / 1e6 * 1.05, C3["executed_ray_steps_per_launch"], 1, None, None)
    assert ok["frac"] is not None and ok["valu_issue"]["frac"] < 1


# ---- post passes: algorithmic bytes against the counted bytes
POST = json.load(open(os.path.join(ROOT, "profiles", "pmc_post.json")))


def _post_key(key):
    which, size = key.rsplit("_", 1)
    W, H = (int(v) for v in size.split("x"))
    return which, W, H


def test_post_counters_present():
    assert {"fxaa_4096x4096", "bloom_4096x4096"} <= set(POST)


@pytest.mark.parametrize("key", sorted(POST))
def test_post_bytes_within_counters(key):
    """No post pass prices more bytes than its kernels move: each kernel's
    algorithmic bytes (bench.post_bytes) and the pass's total stay within 10 %
    of the rocprofv3 HBM bytes of the same kernels (2 FETCH + WRITE)."""
    which, W, H = _post_key(key)
    b = bench.post_bytes(W, H, which)
    c = POST[key]
    assert set(b["kernels"]) == set(c["kernels"]), (b["kernels"], c["kernels"])
    for k, v in b["kernels"].items():
        assert v <= 1.1 * c["kernels"][k], (key, k, v, c["kernels"][k])
    assert b["total"] <= 1.1 * c["hbm_bytes"]


def test_post_line_fracs_below_peak():
    counters = {"bloom_4096x4096": POST["bloom_4096x4096"]}
    line = bench._post_line("bloom", 0.05, 4096, 4096, "bloom", counters)
    assert line["algorithmic_bytes"] == bench.post_bytes(4096, 4096, "bloom")["total"]
    assert line["frac"] < 1 and line["counter_frac"] < 1
    assert line["traffic"] == POST["bloom_4096x4096"]["hbm_bytes"]


def test_post_bytes_model():
    P = bench.post_plan(4096, 4096)
    assert (P["d1"], P["d2"], P["pyramid"]) == (7, 8, True)
    px = 4 * 4096 * 4096
    bl, ch = bench.post_bytes(4096, 4096, "bloom"), bench.post_bytes(4096, 4096, "chain")
    # bloom of a frame reads it twice (pyramid, base texel) and writes it once;
    # the chain is FXAA's frame in and out plus bloom of it
    assert 3 * px < bl["total"] < 3.05 * px
    assert ch["total"] == bench.post_bytes(4096, 4096, "fxaa")["total"] + bl["total"]
    # lod <= 0: one kernel, frame in and out
    assert bench.post_bytes(64, 16, "bloom")["kernels"] == {"bloom": 2 * 4 * 64 * 16}


def test_pmc_of_another_build_nulls_frac_on_every_path():
    """Counters tagged with another build's render code hash price no launch:
    not the counted frame, not a rank's share, not a walk."""
    pmc = dict(C3, render_code_hash="0123456789abcdef")
    ms = C3["avg_kernel_ns_trace"] / 1e6
    for exact in (True, False):
        r = bench.roofline(pmc, ms, C3["executed_ray_steps_per_launch"] // 2, 0, None, None, exact=exact,
                           rows_frac=0.5, code_hash="fedcba9876543210")
        assert r["frac"] is None and "render code" in r["frac_null_reason"]
    # the same hash (or none recorded) prices as before
    r = bench.roofline(pmc, ms, C3["executed_ray_steps_per_launch"], 0, None, None, code_hash="0123456789abcdef")
    assert r["frac"] is not None
