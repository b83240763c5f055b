"""bench.py's balanced split: the runs it derives from one
timed exchange of the even split.  Pure host logic, CPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import balanced_runs  # noqa: E402


def test_link_bound_gives_the_root_a_longer_run():
    # N = 2, C3-like: render halves 0.233 ms, gather 0.39 ms through one link
    runs, m = balanced_runs(2, 16, 4096, {"render_ms": [0.233, 0.233], "gather_ms": 0.39, "deinterleave_ms": 0.02})
    assert runs[1] == 16 and runs[0] > 16
    # rank 0 busy (s0 T1 + d) equals the others' (s max(T1, G)) at the model's shares
    T1, G = 0.466, 0.78
    assert abs((m["share_root"] * T1 + 0.02) - m["share_other"] * max(T1, G)) < 1e-9
    assert abs(m["share_root"] + m["share_other"] - 1.0) < 1e-9


def test_compute_bound_root_takes_a_little_less_for_its_deinterleave():
    runs, _ = balanced_runs(8, 16, 4096, {"render_ms": [0.07] * 8, "gather_ms": 0.001, "deinterleave_ms": 0.02})
    assert runs[0] < 16 and runs[1:] == [16] * 7


def test_root_run_is_capped_so_every_rank_keeps_rows():
    runs, _ = balanced_runs(2, 16, 512, {"render_ms": [0.1, 0.1], "gather_ms": 50.0, "deinterleave_ms": 0.1})
    assert runs[0] == 512 // 2 - 16 and sum(runs) <= 512 // 2


def test_compressed_wire_root_decode_shortens_the_root_run():
    """The compressed wire's exchange (round 6, profiles/r06/scale_model_*):
    at N = 8 the other ranks' messages cross in ~0.013 ms, and the root's
    0.04 ms decode of the seven parts is its extra work, so its run shrinks
    well below a band (the scale model's balanced run was 9 of 16)."""
    runs, m = balanced_runs(8, 16, 4096, {"render_ms": [0.075] * 8, "gather_ms": 0.013, "deinterleave_ms": 0.04})
    assert 4 <= runs[0] <= 11 and runs[1:] == [16] * 7, runs
    assert m["share_root"] < m["share_other"]


def test_wire_defaults_to_the_trial_of_both():
    """bench.py's defaults for N > 1: both splits and both wires in the
    untimed trial (--balance auto --wire auto)."""
    import bench
    src = open(bench.__file__).read()
    assert 'ap.add_argument("--wire", default="auto"' in src
    assert 'ap.add_argument("--balance", default="auto"' in src
