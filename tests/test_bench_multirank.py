"""bench.py end to end, small: the frame check (the timed kernel's last frame
equals the instrumented kernel's, bit for bit) and, for N > 1 ranks, the
exchange figures the scaling run reports (gather_ms, deinterleave_ms,
kernel_ms per rank).  N = 2 with the gloo backend is the one-GPU rehearsal of
the multi-rank path (two ranks on device 0, host-staged gather); the RCCL
("nccl") run needs two GPUs and is skipped below that."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "3", "--warmup", "1", "--spinup", "0", "--size", "512", "--cpu-seconds", "0"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-3000:])
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _rates_within_peak(d):
    """Every achieved rate of the line is at most its peak, and frac is never
    the instrumented tally's (PMC-priced, or null with a reason)."""
    if isinstance(d, dict):
        if d.get("achieved") is not None and d.get("peak"):
            assert d["achieved"] <= d["peak"], d
        for v in d.values():
            _rates_within_peak(v)


def _check_roofline(res):
    roof = res["roofline"]
    _rates_within_peak(res)
    assert "reference_equivalent_tflops" not in roof and "tally_tflops" not in roof, roof
    if roof["frac"] is None:
        assert roof["frac_null_reason"], roof
    else:
        assert "PMC" in roof["flop_source"] and roof["frac"] < 1, roof


def _torchrun(n, extra):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(n)] + extra


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["T", "O"])
def test_bench_one_gpu_frame_check(torch_cuda, scene):
    res = _run([sys.executable, "bench.py"] + SMALL + ["--scene", scene])
    assert res["frame_check"]["result"] == "bit-exact" and res["frame_check"]["pixels"] == 512 * 512, res
    assert res["n_gpus"] == 1 and "gather_ms" not in res
    _check_roofline(res)
    assert res["roofline"]["frac"] is None  # no counters for a 512x512 frame
    # the reference's whole frame (render -> FXAA -> bloom of the FXAA frame),
    # its post chain checked against rm_fxaa then rm_bloom
    assert res["pipeline"]["chain_check"]["result"] == "bit-exact", res["pipeline"]
    assert res["pipeline_ms"] > 0 and res["pipeline"]["post_chain"]["ms"] > 0, res


@pytest.mark.gpu
def test_bench_two_ranks_gloo_rehearsal(torch_cuda):
    """Two ranks on one GPU over gloo: the whole multi-rank path of bench.py
    (row bands, RGB8 wire, gather, de-interleave) and its exchange figures."""
    res = _run(_torchrun(2, SMALL + ["--backend", "gloo", "--balance", "even", "--wire", "rgb8"]))
    assert res["n_gpus"] == 2 and res["frame_check"]["result"] == "bit-exact", res
    assert len(res["kernel_ms_per_rank"]) == 2 and all(k > 0 for k in res["kernel_ms_per_rank"]), res
    assert res["gather_ms"] > 0 and res["deinterleave_ms"] > 0 and res["backend"] == "gloo", res
    assert res["root_ingress_bytes"] == 256 * 3 * 512 and res["wire_bytes_per_rank"] == [256 * 3 * 512] * 2, res
    assert res["balance"] == {"mode": "even", "chosen": "even/rgb8", "runs": [16, 16], "wire": "rgb8"}, res
    _check_roofline(res)
    assert len(res["roofline"]["per_rank_frac"]) == 2 and res["roofline"]["rank"] in (0, 1), res
    assert sum(res["executed_ray_steps_per_rank"]) == res["config"]["executed_ray_steps_per_frame"], res


@pytest.mark.gpu
def test_bench_two_ranks_gloo_balanced(torch_cuda):
    """--balance auto: the host-staged gloo gather is slow, so the balanced
    split (rank 0 renders a longer run of every cycle) is sized from the timed
    exchange, wins the trial, and its frame is still bit-exact."""
    res = _run(_torchrun(2, SMALL + ["--backend", "gloo", "--balance", "auto", "--wire", "rgb8"]))
    b = res["balance"]
    assert b["chosen"] == "balanced/rgb8" and b["balanced_runs"][0] > 16 and b["balanced_runs"][1] == 16, res
    assert res["frame_check"]["result"] == "bit-exact", res
    runs = b["runs"]
    cyc = sum(runs)
    n1 = (512 // cyc) * runs[1] + min(max(512 % cyc - runs[0], 0), runs[1])
    assert res["root_ingress_bytes"] == n1 * 3 * 512 and sum(res["wire_bytes_per_rank"]) == 512 * 3 * 512, res


@pytest.mark.gpu
def test_bench_two_ranks_gloo_compressed_wire(torch_cuda):
    """--wire delta: the compressed wire (DeltaFrame) end to end, bit-exact,
    with fewer bytes into the root than the RGB8 wire's."""
    res = _run(_torchrun(2, SMALL + ["--backend", "gloo", "--balance", "even", "--wire", "delta"]))
    assert res["balance"]["chosen"] == "even/delta" and res["wire"] == "delta", res
    assert res["frame_check"]["result"] == "bit-exact", res
    assert 0 < res["root_ingress_bytes"] < 256 * 3 * 512, res


@pytest.mark.gpu
def test_bench_two_ranks_gloo_default_tries_both_wires(torch_cuda):
    """The default (--balance auto --wire auto): the even and balanced RGB8
    plans and the compressed wire all run untimed trial frames, the fastest
    is timed, and its frame is bit-exact."""
    res = _run(_torchrun(2, SMALL + ["--backend", "gloo"]))
    b = res["balance"]
    assert {"even/rgb8", "even/delta"} <= set(b["trial_ms"]), b
    assert b["chosen"] == min(b["trial_ms"], key=b["trial_ms"].get) and res["wire"] == b["wire"], b
    assert res["frame_check"]["result"] == "bit-exact", res


@pytest.mark.gpu
def test_bench_two_gpus_rccl(torch_cuda):
    """The same over RCCL, one rank per GPU (skipped below two GPUs)."""
    if torch_cuda.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    res = _run(_torchrun(2, SMALL))
    assert res["n_gpus"] == 2 and res["frame_check"]["result"] == "bit-exact", res
    assert res["gather_ms"] > 0 and res["deinterleave_ms"] > 0 and res["backend"] == "nccl", res
