#!/usr/bin/env python3
"""bench.py -- ray-steps/s and frames/s of the HIP ray-march pass on MI355X.

Workload (BASELINE.json metric "ray-steps/sec + frames/sec at 4096x4096,
1/2/4/8 MI355X"): config C3/C4 -- a 4096x4096 frame of scene T (the repaired
template.frag: Menger sponge, castRay + reflection march + AO + soft shadow),
256 max steps, reference start pose P0.  One step = one frame: every rank
renders its row bands (rows dealt in bands of 16, round robin), packs them to
RGBA8 (the reference's RenderTexture format), and for N > 1 one RCCL gather
brings them to rank 0, which de-interleaves the frame.  Total work per step is
fixed as N grows (strong scaling).  The inputs are uniforms only (synthetic:
the pose), nothing is read from the host inside the timed region.

Tiles are dispatched costliest first (rm_params.schedule, the default): each
launch's tile durations order the next launch of the same geometry, so every
timed frame uses the order measured on the frame before it (the first, untimed
launches run row-major); --schedule rowmajor turns it off.

value = sceneSDF evaluations (ray-steps) of one frame x steps / wall time of
the timed region (max over ranks).  The per-frame step count comes from one
instrumented run of the same kernel (count_evals) before timing; the timed
runs are uninstrumented.

--walk measures under the reference's operating condition instead of a still
camera: every frame moves the camera one step forward as main.cpp does with W
held (pos += dir * 0.1 along the view-rotated axes, main.cpp:153-171) and
advances u_time by the 60 Hz frame interval (main.cpp:30,190-191), which
rotates the sponge.  The warm-up frames walk up to the start pose, the timed
frames walk on from it (deterministic poses; their ray-steps are counted by an
instrumented pass over the same poses before timing).

Usage: python bench.py [--gpus N --steps K --warmup W] [--scene T|O|S0]
       [--size 4096] [--max-steps 256] [--pose P0] [--band 16] [--walk]
       [--fmt rgba8|float4] [--kernel auto|tile16|tile8] [--cpu-seconds 12]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0     # HBM3E spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--spinup", type=float, default=0.3,
                    help="seconds of untimed frames before the warm-up frames (GPU clock ramp)")
    ap.add_argument("--scene", default="T")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--max-steps", type=int, default=256)
    ap.add_argument("--pose", default="P0")
    ap.add_argument("--band", type=int, default=16)
    ap.add_argument("--balance", default="auto", choices=["auto", "even"],
                    help="N > 1: 'even' deals rows in round-robin bands of --band; 'auto' also measures a "
                         "split that gives rank 0 (which receives every other rank's rows and de-interleaves) "
                         "a longer run per cycle, sized from the timed exchange, and keeps whichever plan ran "
                         "the untimed trial frames faster")
    ap.add_argument("--wire", default="auto", choices=["auto", "rgb8", "delta"],
                    help="N > 1: the RGB8 wire (3 B/px), the compressed wire (DeltaFrame: the render kernel "
                         "encodes its 8x8 tiles losslessly, ~7x fewer bytes on C3, DESIGN.md 4.4), or 'auto' "
                         "(default): both in the untimed trial, the faster timed")
    ap.add_argument("--chunks", type=int, default=None,
                    help="render/gather chunks per frame (default 1: frames are pipelined instead)")
    ap.add_argument("--fmt", default="rgba8", choices=["rgba8", "float4"])
    ap.add_argument("--streams", type=int, default=None, choices=[1, 2],
                    help="HIP streams frames alternate on (default: 2 for N > 1 over RCCL, else 1; at N = 1 "
                         "two streams measure the same C3 frame time (0.4218-0.4220 against 0.4180-0.4225 ms, "
                         "profiles/r05/n1_streams), and each launch then overlaps the next, so rocprofv3's "
                         "per-launch durations no longer equal the kernel's)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "tile16", "tile8"])
    ap.add_argument("--schedule", default="adaptive", choices=["adaptive", "rowmajor"],
                    help="tile dispatch order: costliest tiles of the previous frame first, or row-major")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse on one GPU)")
    ap.add_argument("--dist-timeout", type=float, default=180.0,
                    help="N > 1: seconds any one collective may take before the run fails (init_process_group timeout)")
    ap.add_argument("--walk", action="store_true",
                    help="moving camera and advancing u_time (main.cpp's W key at 60 Hz) instead of a still pose")
    ap.add_argument("--walk-speed", type=float, default=0.1, help="camera step per frame (main.cpp:21 speed)")
    ap.add_argument("--walk-dt", type=float, default=1.0 / 60.0, help="u_time step per frame (main.cpp:30)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--post-pmc", default=os.path.join(HERE, "profiles", "pmc_post.json"),
                    help="per post pass rocprofv3 HBM bytes (tools/make_post_traffic.py)")
    ap.add_argument("--pmc", default=os.path.join(HERE, "profiles", "pmc_counters.json"),
                    help="per-workload rocprofv3 PMC counters (profiles/): executed FP32 ops for "
                         "roofline.achieved, HBM bytes for roofline.traffic, VALU/SALU issue")
    return ap.parse_args()


def _config_id(scene, W, H, max_steps, world):
    """SURVEY.md 8(d) config name for a workload; "custom" when it matches none."""
    if scene == "S0" and (W, H) == (256, 256):
        return "C1"
    if scene == "T" and (W, H, max_steps) == (1920, 1080, 128):
        return "C2"
    if scene == "T" and (W, H, max_steps) == (4096, 4096, 256):
        return "C3" if world == 1 else "C4"
    if scene == "O" and (W, H, max_steps) == (8192, 8192, 512):
        return "C5"
    return "custom"


def walk_pose(pose, i, speed, dt):
    """Frame i of a walk from `pose` (i < 0: the frames before it): main.cpp's
    camera step with W held, pos += dir * speed with dir = (0, 0, -1) rotated by
    the pose's mouse angles (YZ by -my, then XZ by mx, main.cpp:155-171), and
    u_time advanced by dt per frame (main.cpp:190-191)."""
    import math

    mx, my = pose["mouse"]
    dty, dtz = math.sin(-my), -math.cos(-my)        # rotate YZ: dir = (0, 0, -1)
    dx, dz = -dtz * math.sin(mx), dtz * math.cos(mx)  # rotate XZ
    px, py, pz = pose["pos"]
    return dict(pos=(px + dx * speed * i, py + dty * speed * i, pz + dz * speed * i), mouse=pose["mouse"],
                time=pose["time"] + dt * i)


def cpu_baseline(args, pose, W, H, target_s):
    """Oracle (CPU restatement, -O3 build) on a strided row sample of the same frame."""
    import oracle  # test infrastructure: only the cpu_baseline leg uses it
    import numpy as np

    L = oracle.lib(fast=True)
    kw = dict(pos=pose["pos"], mouse=pose["mouse"], time=pose["time"], max_steps=args.max_steps)
    # calibrate on 8 evenly spread rows, then size the sample to ~target_s
    probe = np.linspace(0, H - 1, 8).astype(np.int32)
    t0 = time.perf_counter()
    oracle.render_rows(args.scene, W, H, probe, fast=True, **kw)
    per_row = (time.perf_counter() - t0) / len(probe)
    nrows = int(max(8, min(H, target_s / max(per_row, 1e-6))))
    stride = max(1, H // nrows)
    rows = np.arange(0, H, stride, dtype=np.int32)
    t0 = time.perf_counter()
    _, ev = oracle.render_rows(args.scene, W, H, rows, fast=True, **kw)
    dt = time.perf_counter() - t0
    evals = int(ev.sum(dtype=np.uint64))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = int(L.oracle_num_threads())
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    omp_env = os.environ.get("OMP_NUM_THREADS")
    return {
        "value": evals / dt,
        "unit": "ray-steps/s",
        "frames_per_s": (len(rows) / H) / dt,
        "cores": threads,
        "kind": "port",
        "threads": {"openmp_threads_used": threads, "OMP_NUM_THREADS": omp_env, "sched_affinity_cpus": affinity,
                    "nproc": os.cpu_count(),
                    "note": "OpenMP runs OMP_NUM_THREADS threads when it is set (the GPU pool sets it to the "
                            "per-GPU CPU share and asks runs to keep it), else one per CPU of the affinity mask; "
                            "nproc counts the whole host"},
        "sample": f"rows y = 0 mod {stride} of the {W}x{H} frame ({len(rows)} rows, {evals} ray-steps, "
                  f"{dt:.2f} s); frames/s extrapolated by row fraction; OpenMP dynamic rows, -O3 "
                  f"x86-64-v3; host CPU: {model}, {threads} threads",
    }


def frame_check(r, frame, W, H, fmt):
    """The last timed frame (rank 0's whole frame: de-interleaved for N > 1)
    against one render of the same pose by the instrumented kernel
    (count_evals=1: every reference ray-step, the kernel the parity tests check
    against the oracle).  The timed kernels leave out steps that cannot change
    the frame (common.frag:810-831, :931-954, :991-1002),
    so the two frames must be the same bits; anything else fails the run."""
    import torch

    timed = frame
    r.set_params(count_evals=1)
    ref = r.render_rgba8(W, H) if fmt == "rgba8" else r.render(W, H)
    r.set_params(count_evals=0)
    torch.cuda.synchronize()
    diff = (timed.view(torch.int32) != ref.view(torch.int32)).reshape(H * W, -1).any(-1)
    nd = int(diff.sum())
    res = {"result": "bit-exact" if nd == 0 else "MISMATCH", "pixels": W * H, "pixels_differing": nd,
           "against": "one render of the last timed pose by the instrumented kernel (count_evals=1, every "
                      "reference ray-step), " + ("RGBA8 words" if fmt == "rgba8" else "float4 bits")}
    if nd:
        print(json.dumps({"frame_check": res}), file=sys.stderr, flush=True)
        raise SystemExit(f"frame_check: {nd} of {W * H} pixels of the timed frame differ from the instrumented frame")
    return res


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def post_plan(W, H):
    """bloom's level pair and passes as rm_post.hip's bloom_plan computes them
    (lod = log2(0.05 H) in float32, levels d1 = floor(lod), d2 = d1 + 1), and
    which mip path a W x H frame takes: the exact-halving pyramid from level
    s0 (W, H multiples of 2^d2, 5..8 levels), per-level resamples otherwise."""
    import numpy as np

    q = max(W, H).bit_length() - 1
    lod = float(np.log2(np.float32(0.05) * np.float32(H)))
    d1 = d2 = 0
    if lod > 0:
        d1 = min(int(np.floor(lod)), q)
        d2 = min(d1 + 1, q)
    w, h = [W], [H]
    for _ in range(d2):
        w.append(max(w[-1] >> 1, 1))
        h.append(max(h[-1] >> 1, 1))
    T2 = 1 << d2
    div = W % T2 == 0 and H % T2 == 0
    s0 = max(d2 - 8, 0)
    pyramid = lod > 0 and d2 - s0 >= 5 and div
    nruns = [min(n, 5 * lw + 1) for n, lw in ((W, w[d1]), (H, h[d1]), (W, w[d2]), (H, h[d2]))] if lod > 0 else []
    return dict(lod=lod, d1=d1, d2=d2, w=w, h=h, s0=s0, pyramid=pyramid, nruns=nruns)


def post_bytes(W, H, which):
    """Algorithmic HBM bytes of one post pass over a W x H RGBA8 frame, per
    kernel: what each kernel must read and write once (re-reads served by the
    caches not counted).  which: "fxaa" (rm_fxaa), "bloom" (rm_bloom of a
    frame), "chain" (rm_post_chain: FXAA then bloom of its output).
      fxaa       the frame in, the frame out (4 + 4 B/px); in the chain also
                 mip level 3 out (4 B per 8 x 8 block)
      mips       the level the pyramid starts from in (the frame: s0 = 0;
                 level 3 in the chain), levels d1 and d2 out; without the
                 pyramid every level 1..d2 out and its parent in
      poly       levels d1, d2 in, the run-pair polynomials out (48 B a pair)
      bloom_min  the frame in and out, the polynomials and the per-column /
                 per-row run entries (24 B each) in
    The run tables (rm_bloom_runs_kernel) depend on W x H only and are built
    once per size, outside the per-frame bytes."""
    P = post_plan(W, H)
    px = 4 * W * H
    k = {}
    if which in ("fxaa", "chain"):
        k["fxaa"] = 2 * px
    if which == "fxaa":
        return dict(kernels=k, total=sum(k.values()), plan=P)
    if P["lod"] <= 0:
        k["bloom"] = 2 * px
        return dict(kernels=k, total=sum(k.values()), plan=P)
    w, h, d1, d2 = P["w"], P["h"], P["d1"], P["d2"]
    lv = lambda j: 4 * w[j] * h[j]  # noqa: E731
    if P["pyramid"]:
        s0 = P["s0"]
        k["mips"] = sum(lv(j - 1) + lv(j) for j in range(1, s0 + 1)) + lv(s0) + lv(d1) + lv(d2)
    else:
        k["mips"] = sum(lv(j - 1) + lv(j) for j in range(1, d2 + 1))
    nr = P["nruns"]
    tabs = 48 * (nr[0] * nr[1] + nr[2] * nr[3])
    k["poly"] = lv(d1) + lv(d2) + tabs
    k["bloom_min"] = 2 * px + tabs + 24 * (W + H)
    return dict(kernels=k, total=sum(k.values()), plan=P)


def load_post_counters(path):
    """profiles/pmc_post.json (tools/make_post_traffic.py): per post pass and
    frame size, the rocprofv3 HBM bytes of one pass, (2 FETCH_SIZE +
    WRITE_SIZE) per kernel launch summed over the pass's kernels."""
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return {}


def _post_line(name, ms, W, H, which, counters):
    b = post_bytes(W, H, which)
    gbs = b["total"] / (ms / 1e3) / 1e9
    line = {"name": name, "ms": ms, "bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": gbs / PEAK_HBM_GBS, "algorithmic_bytes": b["total"], "algorithmic_bytes_per_kernel": b["kernels"],
            "traffic": None, "counter_frac": None}
    c = counters.get(f"{which}_{W}x{H}")
    if c:
        line.update(traffic=c["hbm_bytes"], counter_frac=c["hbm_bytes"] / (ms / 1e3) / 1e9 / PEAK_HBM_GBS,
                    traffic_per_kernel=c.get("kernels"), traffic_source=c.get("source"),
                    traffic_note="rocprofv3 (2 FETCH_SIZE + WRITE_SIZE) per pass, profiles/pmc_post.json")
    return line


def _timed(stream, reps, fn):
    import torch

    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def time_fxaa(r, frame8, stream, counters, reps=20):
    """The reference's FXAA pass (post.frag) over the RGBA8 frame on rank 0:
    HBM-bound stencil, 4 B read + 4 B written per pixel (algorithmic)."""
    import torch

    H, W = frame8.shape
    out = torch.empty_like(frame8)
    ms = _timed(stream, reps, lambda: r.fxaa(frame8, out=out))
    return _post_line("fxaa (post.frag:16-61,135-144)", ms, W, H, "fxaa", counters)


# per pixel (rm_post.hip rm_bloom_min_kernel): the base-level bilinear fetch
# (27), per level and channel the run pair's bilinear polynomial (3 multiply-adds,
# 2 levels x 3 channels), the level sum (3), threshold and add (9).  The run-pair
# polynomials (25 taps each, double) are per frame, ~1e-3 of this at 4096^2.
BLOOM_FLOP_PER_PX = 27 + 2 * 3 * 3 * 2 + 3 + 9


def time_bloom(r, frame8, stream, counters, reps=20):
    """The reference's bloom pass (bloom.frag + its mip chain, main.cpp:212-214)
    over an RGBA8 frame on rank 0, priced by the bytes its kernels move
    (post_bytes "bloom"); per pixel two bilinear polynomials
    (BLOOM_FLOP_PER_PX) are reported beside it."""
    import torch

    H, W = frame8.shape
    out = torch.empty_like(frame8)
    ms = _timed(stream, reps, lambda: r.bloom(frame8, out=out))
    line = _post_line("bloom (shaders/post/bloom.frag:14-43 + mip chain)", ms, W, H, "bloom", counters)
    tflops = W * H * BLOOM_FLOP_PER_PX / (ms / 1e3) / 1e12
    line.update(mip_levels=post_plan(W, H)["d2"],
                valu={"flop_per_px": BLOOM_FLOP_PER_PX, "achieved": tflops, "peak": PEAK_FP32_TFLOPS,
                      "unit": "TFLOP/s", "frac": tflops / PEAK_FP32_TFLOPS})
    return line


def time_pipeline(r, W, H, stream, counters, render_ms, reps=20):
    """The reference's whole frame (main.cpp:196-214) on rank 0: the ray-march
    pass into the RGBA8 frame, FXAA into postTexture, its mip chain and bloom of
    it into the output (rm_post_chain), frame after frame on one stream.
    pipeline_ms = event interval per frame; post_chain = the two post passes
    alone; chain_check: rm_post_chain's output against rm_fxaa then rm_bloom of
    the same frame (GPU, bit for bit; tests/test_post_chain.py holds the
    oracle's chain).  Untimed frames for 0.3 s first, as before the timed
    frames."""
    import torch

    frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
    mid, out = torch.empty_like(frame), torch.empty_like(frame)

    def step():
        r.render_rgba8(W, H, out=frame)
        r.post_chain(frame, mid=mid, out=out)

    import time
    t_end = time.time() + 0.3  # spin-up as for the timed frames: the GPU's clocks settle to the mixed load
    while time.time() < t_end:
        step()
        stream.synchronize()
    pipe_ms = _timed(stream, reps, step)
    chain_ms = _timed(stream, reps, lambda: r.post_chain(frame, mid=mid, out=out))
    ref = r.bloom(r.fxaa(frame))
    torch.cuda.synchronize()
    nd = int((ref != out).sum())
    chain = _post_line("post chain: fxaa + mips + bloom (main.cpp:209-214, rm_post_chain)", chain_ms, W, H, "chain",
                       counters)
    return {"pipeline_ms": pipe_ms, "pipeline_frames_per_s": 1e3 / pipe_ms,
            "render_ms": render_ms, "post_chain": chain,
            "chain_check": {"result": "bit-exact" if nd == 0 else "MISMATCH", "pixels_differing": nd,
                            "against": "rm_fxaa then rm_bloom of the last frame"},
            "note": "render (adaptive order, as the timed frames) -> FXAA -> mip chain -> bloom of the FXAA frame, "
                    f"{reps} frames back to back on one stream, HIP events around them; render_ms = the timed "
                    "frames' ms_per_step"}


def balanced_runs(world, band, H, ex):
    """Rows per cycle for each rank from one even-split timed exchange, per-rank
    lists of render_ms / pack_ms and rank 0's gather_ms / deinterleave_ms.
    With every rank rendering 1/N of the rows, the frame costs T1 = sum of the
    renders on one GPU and G = N * gather_ms to move whole through one link
    (each non-root rank's rows cross their own xGMI link, concurrently).  A
    non-root rank with share s is busy s * max(T1, G) per pipelined frame (its
    render and its send overlap); rank 0 is busy s0 * T1 + de-interleave, with
    s0 = 1 - (N - 1) s.  Equal busy times give
        s = (T1 + d) / (max(T1, G) + (N - 1) T1),
    and rank 0's run is band * s0 / s (the others keep `band`), capped so that a
    cycle fits twice in the frame (every rank keeps rows)."""
    T1 = sum(ex["render_ms"])
    G = world * ex["gather_ms"]
    d = ex["deinterleave_ms"]
    s = (T1 + d) / (max(T1, G) + (world - 1) * T1)
    s0 = max(1.0 - (world - 1) * s, 0.0)
    r0 = int(min(max(round(band * s0 / s), 1), max(1, H // 2 - (world - 1) * band)))
    return [r0] + [band] * (world - 1), dict(T1_ms=T1, G_ms=G, deinterleave_ms=d, share_other=s, share_root=s0)


_F32_KEYS = ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F32")


def pmc_flop(pmc):
    """(FP32 FLOP done by active lanes in one PMC-counted launch, issued lane
    slots, active-lane fraction), or None without the F32 counters:
    64 x (ADD + MUL + TRANS + 2 FMA) wave-instructions, scaled by the mean
    active-lane fraction SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)."""
    if not all(k in pmc for k in _F32_KEYS):
        return None
    slots = 64 * (pmc[_F32_KEYS[0]] + pmc[_F32_KEYS[1]] + pmc[_F32_KEYS[2]] + 2 * pmc[_F32_KEYS[3]])
    lane_frac = pmc.get("active_lane_frac")
    return slots * (lane_frac or 1.0), slots, lane_frac


# a PMC entry counts this build's launch only if its traced duration is within this ratio of the measured one
PMC_TIME_TOL = (0.9, 1.1)


def pmc_build_mismatch(pmc, code_hash):
    """Why a PMC entry does not count this build's render launch, or None: its
    render_code_hash (tools/make_traffic_json.py) differs from the loaded
    library's rm_render_code_hash().  Entries without a hash (older profiles)
    are checked by launch duration only (roofline)."""
    h = pmc.get("render_code_hash") if pmc else None
    if h and code_hash and h != code_hash:
        return (f"the PMC counters in profiles/pmc_counters.json ({pmc.get('source')}) were taken with render code "
                f"{h}, this library's is {code_hash}")
    return None


def roofline(pmc, kern_ms, executed_steps, out_bytes, flop_tally, evals, exact=True, rows_frac=1.0, code_hash=None):
    """The render kernel's FP32-VALU roofline for one launch of kern_ms that
    executed `executed_steps` ray-steps and wrote out_bytes.

    pmc holds rocprofv3 --pmc counters (profiles/pmc_counters.json) of one N = 1
    launch.  exact: they are counters of this very workload (same frame, pose,
    build): FLOP = the counted FLOP.  Otherwise (a rank's share of that frame
    for N > 1, or a walk): FLOP = executed_steps x (the counted FLOP / the
    counted launch's executed ray-steps), and the HBM traffic = the counted
    traffic x rows_frac.  With no counters the FP32 FLOP are not known and frac
    is null with the reason: the instrumented per-term tally (SURVEY.md 8(d)
    prices over the terms evaluated, incl. work exact exits skip) is reported as
    tally_frac only, never as frac."""
    if not kern_ms or kern_ms <= 0:  # a rank with no rows launches nothing
        return {"bound": "valu", "achieved": None, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": None,
                "traffic": None, "frac_null_reason": "no launch (no rows on this rank)"}
    t = kern_ms / 1e3
    cnt = pmc_flop(pmc) if pmc else None
    base_steps = pmc.get("executed_ray_steps_per_launch") if pmc else None
    stale = pmc_build_mismatch(pmc, code_hash)  # (every path: exact, a rank's share, a walk)
    if stale:
        cnt = None
    if not stale and exact and pmc and pmc.get("avg_kernel_ns_trace"):
        # counters of another build: the profiled launch's duration is off this one's by > 10 %
        ratio = kern_ms * 1e6 / pmc["avg_kernel_ns_trace"]
        if not PMC_TIME_TOL[0] <= ratio <= PMC_TIME_TOL[1]:
            stale = (f"the PMC counters in profiles/pmc_counters.json ({pmc.get('source')}) are stale: their launch "
                     f"took {pmc['avg_kernel_ns_trace'] / 1e6:.4g} ms, this one {kern_ms:.4g} ms")
            cnt = None
    roof = {"bound": "valu", "achieved": None, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": None,
            "traffic": None, "flop_per_launch": None, "executed_ray_steps_per_launch": executed_steps,
            "ray_steps_per_launch": evals, "kernel_ms": kern_ms}
    if cnt is not None and (exact or base_steps):
        flop_c, slots, lane_frac = cnt
        if exact:
            flop = flop_c
            src = (f"PMC executed FP32 ops of this workload ({pmc.get('source')}): 64 x (ADD + MUL + TRANS + 2 FMA)"
                   + (" x active-lane fraction" if lane_frac else " (issued lane slots)"))
        else:
            per_step = flop_c / base_steps
            flop = executed_steps * per_step
            slots = slots * executed_steps / base_steps
            src = (f"this launch's executed ray-steps x the PMC FP32 FLOP per executed ray-step of the N = 1 launch "
                   f"of the same workload ({pmc.get('source')}: {flop_c:.4g} FLOP / {base_steps} steps = "
                   f"{per_step:.2f})")
        ach = flop / t / 1e12
        roof.update(achieved=ach, frac=ach / PEAK_FP32_TFLOPS, flop_per_launch=flop, flop_source=src,
                    active_lane_frac=lane_frac, issued_lane_slot_frac=slots / t / 1e12 / PEAK_FP32_TFLOPS)
        if pmc.get("hbm_bytes_per_launch") is not None:
            roof["traffic"] = pmc["hbm_bytes_per_launch"] * (1.0 if exact else rows_frac)
    else:
        roof["frac_null_reason"] = stale or (
            "no PMC counters for this workload in profiles/pmc_counters.json" if cnt is None else
            "the PMC entry of this workload has no executed_ray_steps_per_launch to price a share of it")
    roof["tally_flop_per_launch"] = flop_tally
    roof["tally_frac"] = None if flop_tally is None else flop_tally / t / 1e12 / PEAK_FP32_TFLOPS
    roof["tally_note"] = ("SURVEY 8(d) per-term price list over the reference terms the instrumented kernel "
                          "evaluates; not executed FP32 FLOP (abs/min/max are free modifiers or med3), not the "
                          "roofline figure")
    gbs = out_bytes / t / 1e9
    roof["hbm"] = {"achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                   "algorithmic_bytes_per_launch": out_bytes, "counter_gbs": None, "counter_frac": None}
    if roof["traffic"] is not None:
        cg = roof["traffic"] / t / 1e9
        roof["hbm"].update(counter_gbs=cg, counter_frac=cg / PEAK_HBM_GBS,
                           counter_note="rocprofv3 (2 FETCH_SIZE + WRITE_SIZE) per launch"
                                        + ("" if exact else " of the N = 1 frame x this launch's row fraction")
                                        + " / kernel_ms")
    if exact and pmc and "SQ_INSTS_VALU" in pmc and not stale:
        # issue fractions at the clock the PMC run measured (GRBM_GUI_ACTIVE / 8 XCDs / kernel time):
        # one wave64 VALU instruction per 2 cycles per SIMD (1024 SIMDs), one SALU per cycle per CU (256)
        clk = pmc.get("clock_hz") or 2.4e9
        roof["valu_issue"] = {"insts_per_launch": pmc["SQ_INSTS_VALU"],
                              "frac": pmc["SQ_INSTS_VALU"] * 2 / (t * clk * 1024), "clock_hz": clk}
        if "SQ_INSTS_SALU" in pmc:
            roof["salu_issue"] = {"insts_per_launch": pmc["SQ_INSTS_SALU"],
                                  "frac": pmc["SQ_INSTS_SALU"] / (t * clk * 256)}
    return roof


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import raymarching_amd as rm
    from raymarching_amd.frame import DeltaFrame, DistributedFrame

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # (ranks > GPUs only in single-GPU gloo rehearsals)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        # a finite timeout on every collective: a first real RCCL exchange that
        # stalls ends the run non-zero with the watchdog's message (the default
        # would wait 10 min per collective) instead of hanging the driver
        import datetime
        to = datetime.timedelta(seconds=args.dist_timeout)
        if args.backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")  # tear down on timeout
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        else:
            dist.init_process_group("gloo", timeout=to)

    W = args.size
    H = args.height or args.size
    pose = rm.S0_POSE if args.scene == "S0" else rm.POSES[args.pose]
    r = rm.Renderer(local)
    r.load_scene(rm.SCENE_FILES[args.scene])
    r.set_uniform("u_resolution", W, H)
    r.set_pose(pose["pos"], pose["mouse"], pose["time"])
    r.set_params(max_steps=args.max_steps, shadow_max_steps=0, kernel=args.kernel, schedule=args.schedule)
    stream = torch.cuda.current_stream(dev)
    r.set_stream(stream)
    chunks = args.chunks if args.chunks is not None else 1
    fr = DistributedFrame(r, W, H, args.band, rank, world, fmt=args.fmt, chunks=chunks, streams=args.streams)
    red_dev = dev if args.backend == "nccl" else torch.device("cpu")

    def spin_up():
        # a fresh GPU ramps its clocks over the first ~0.1 s of load.  Every rank
        # runs the same number of rounds (each frame holds a gather), so whether
        # to go on is agreed over all ranks after each round.
        t_spin = time.perf_counter()
        while args.spinup > 0:
            for _ in range(8):
                fr.submit()
            fr.flush()
            torch.cuda.synchronize(dev)
            go = torch.tensor([1.0 if time.perf_counter() - t_spin < args.spinup else 0.0], device=red_dev)
            if world > 1:
                dist.all_reduce(go, op=dist.ReduceOp.MIN)
            if go.item() == 0.0:
                break

    def trial_ms(f, n=16):
        # untimed trial: pipelined frames, wall time, max over ranks; at least n
        # frames and about 20 ms of them (the count agreed over the ranks from
        # the warm-up frames: every rank must run the same collectives)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(4):
            f.submit()
        f.flush()
        torch.cuda.synchronize(dev)
        est = torch.tensor([(time.perf_counter() - t0) / 4 * 1e3], dtype=torch.float64, device=red_dev)
        dist.all_reduce(est, op=dist.ReduceOp.MAX)
        n = int(min(256, max(n, math.ceil(20.0 / max(float(est.item()), 1e-3)))))
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(n):
            f.submit()
        f.flush()
        torch.cuda.synchronize(dev)
        dist.barrier()
        tt = torch.tensor([(time.perf_counter() - t1) / n * 1e3], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    balance = None
    if world > 1 and args.fmt == "rgba8" and (args.balance == "auto" or args.wire != "rgb8"):
        # plan calibration (untimed): candidate frames -- the even split over
        # the RGB8 wire, the balanced split its timed exchange implies, the even
        # split over the compressed wire -- each run for trial frames; the
        # fastest is timed
        spin_up()
        cands, errors, runs, model = {}, {}, None, None

        def build(name, make):
            try:
                f = make()
                cands[name] = (f, trial_ms(f))
            except Exception as e:  # noqa: BLE001 -- keep the others; say why in the line (the same on every rank)
                errors[name] = f"{type(e).__name__}: {e}"
                torch.cuda.synchronize(dev)

        def exchange(f):  # the even split's timed exchange, every rank's figures (collective)
            xs = [f.timed_exchange() for _ in range(3)]
            mine = torch.tensor([_median([x[k] for x in xs]) for k in ("render_ms", "pack_ms", "gather_ms",
                                                                        "deinterleave_ms")],
                                dtype=torch.float64, device=red_dev)
            per = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(per, mine)
            per = [[float(v) for v in x.cpu()] for x in per]
            return {"render_ms": [x[0] for x in per], "pack_ms": [x[1] for x in per], "gather_ms": per[0][2],
                    "deinterleave_ms": per[0][3]}

        runs_delta, model_delta = None, None
        if args.wire in ("auto", "rgb8"):
            cands["even/rgb8"] = (fr, trial_ms(fr))
            if args.balance == "auto":
                runs, model = balanced_runs(world, args.band, H, exchange(fr))
                build("balanced/rgb8", lambda: DistributedFrame(r, W, H, args.band, rank, world, fmt=args.fmt,
                                                                chunks=chunks, streams=args.streams, runs=runs))
        if args.wire in ("auto", "delta"):
            build("even/delta", lambda: DeltaFrame(r, W, H, args.band, rank, world, streams=args.streams))
            if args.balance == "auto" and "even/delta" in cands:
                # the root renders rows and decodes every other part: its run
                # sized from the compressed wire's own exchange
                runs_delta, model_delta = balanced_runs(world, args.band, H, exchange(cands["even/delta"][0]))
                if runs_delta != [args.band] * world:
                    build("balanced/delta", lambda: DeltaFrame(r, W, H, args.band, rank, world,
                                                               streams=args.streams, runs=runs_delta))
        chosen = min(cands, key=lambda k: cands[k][1])
        fr = cands[chosen][0]
        balance = {"mode": f"balance {args.balance}, wire {args.wire}", "chosen": chosen,
                   "runs": list(fr.plan.part_runs), "wire": fr.wire,
                   "trial_ms": {k: v[1] for k, v in cands.items()}, "balanced_runs": runs, "model": model,
                   "balanced_runs_delta": runs_delta, "model_delta": model_delta,
                   "note": "untimed trial frames (16-256 pipelined frames per candidate, about 20 ms, max over ranks) before the "
                           "instrumented run and the warm-up; the timed frames use the chosen candidate"}
        if errors:
            balance["errors"] = errors
        cands.clear()
    elif world > 1:
        balance = {"mode": "even", "chosen": "even/" + fr.wire, "runs": [args.band] * world, "wire": fr.wire}

    def set_frame(i):  # walk: the pose of frame i (timed frames 0..K-1)
        if args.walk:
            p = walk_pose(pose, i, args.walk_speed, args.walk_dt)
            r.set_pose(p["pos"], p["mouse"], p["time"])

    # instrumented run: ray-steps of this rank's rows, summed over ranks (with
    # --walk: per timed pose, their mean is the frame's count)
    r.set_params(count_evals=1)
    walk_evals, walk_skipped = [], []
    for i in range(args.steps if args.walk else 1):
        set_frame(i)
        _, st = fr.render_local(stats=True)
        walk_evals.append(st["evals"])
        walk_skipped.append(st.get("skipped", 0))
    if args.walk:
        st = dict(st, evals=sum(walk_evals) / len(walk_evals), skipped=sum(walk_skipped) / len(walk_skipped))
    r.set_params(count_evals=0)
    ev_rank = torch.tensor([st["evals"], st.get("skipped", 0)], dtype=torch.float64, device=red_dev)
    ev_total = ev_rank.clone()
    if world > 1:
        dist.all_reduce(ev_total)
    evals_rank, evals_frame = int(ev_rank[0].item()), int(ev_total[0].item())
    skipped_frame = int(ev_total[1].item())
    exec_rank = evals_rank - int(ev_rank[1].item())  # ray-steps this rank's launch executes
    rank_launch = [dict(kernel_ms=None, executed_steps=exec_rank, rows=fr.nmine)]

    # untimed spin-up before the W warm-up frames: a fresh GPU ramps its clocks
    # over the first ~0.1 s of load (3 warm-up frames are ~3 ms), so the timed
    # frames would otherwise include the ramp.  Same frames, same work.
    set_frame(-args.warmup)
    spin_up()
    for i in range(-args.warmup, 0):
        set_frame(i)
        fr.submit()
    fr.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    nch = len(fr.cuts) - 1
    # frame-stream interval: with one frame stream and one chunk, one event pair
    # on that stream around the whole timed region (per-frame timing events
    # cost 2 % of a C3 frame: 0.481 -> 0.471 ms without them,
    # profiles/r03/bench_events_ab.jsonl); otherwise a pair around each render
    whole = len(fr.streams) == 1 and nch == 1
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nch)]
           for _ in range(1 if whole else args.steps)]
    if whole:
        evs[0][0][0].record(fr.streams[0])
    t0 = time.perf_counter()
    for i in range(args.steps):
        set_frame(i)
        fr.submit(events=None if whole else evs[i])  # frame i's gather overlaps frame i+1's render
    if whole:
        evs[0][0][1].record(fr.streams[0])
    fr.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    last_frame = fr.frame.clone() if fr.frame is not None else None  # the last timed frame (rank 0)
    live = [c for c in range(nch) if min(fr.cuts[c + 1], fr.nmine) > fr.cuts[c]]  # chunks with rows here
    # per-frame interval of the render calls on the frame stream (events around each call: the render
    # kernel plus the dispatch-order sort it enqueues; with 2 streams it also spans overlapping frames)
    if whole:
        frame_stream_ms = evs[0][0][0].elapsed_time(evs[0][0][1]) / args.steps if live else 0.0
    else:
        frame_stream_ms = sum(evs[i][c][0].elapsed_time(evs[i][c][1]) for i in range(args.steps) for c in live) / args.steps
    # per-launch render-kernel duration (the roofline denominator): synchronous launches of this rank's
    # rows on the frames' stream, HIP events around the kernel alone (rm_stats.kernel_ms), after the
    # timed region
    set_frame(args.steps - 1)
    launch = sorted(fr.render_local(stats=True)[1]["kernel_ms"] for _ in range(11)) if fr.nmine else [0.0]
    kern = launch[len(launch) // 2]
    kt = torch.tensor([kern], dtype=torch.float64, device=red_dev)
    # the last timed frame against the instrumented kernel's frame of the same pose (rank 0)
    check = frame_check(r, last_frame, W, H, args.fmt) if rank == 0 else None
    exchange = None
    if world > 1:
        # the frame's steps one at a time (render, pack, gather, de-interleave),
        # each timed alone after the timed region: the gather's own time, which
        # the pipelined frames overlap with the next frame's render
        xs = [fr.timed_exchange() for _ in range(5)]
        wire_row = fr.wires[0].stride(0) * fr.wires[0].element_size()  # bytes of one row on the wire
        if fr.wire == "delta":  # the messages' measured sizes (the last timed exchange)
            wire_sizes = [int(v) for v in xs[-1]["wire_bytes"]]
        else:
            wire_sizes = [fr.plan.count(q) * wire_row for q in range(world)]
        mine = torch.tensor([kern, exec_rank, fr.nmine] + [_median([x[k] for x in xs]) for k in (
            "render_ms", "pack_ms", "gather_ms", "deinterleave_ms")], dtype=torch.float64, device=red_dev)
        per_rank = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
        pr = [[float(v) for v in x.cpu()] for x in per_rank]
        rank_launch = [dict(kernel_ms=x[0], executed_steps=int(x[1]), rows=int(x[2])) for x in pr]
        exchange = {
            "gather_ms": pr[0][5], "deinterleave_ms": pr[0][6], "pack_ms": pr[0][4],
            "kernel_ms_per_rank": [x[0] for x in pr], "gather_ms_per_rank": [x[5] for x in pr],
            "pack_ms_per_rank": [x[4] for x in pr],
            "executed_ray_steps_per_rank": [int(x[1]) for x in pr], "rows_per_rank": [int(x[2]) for x in pr],
            "wire_bytes_per_rank": wire_sizes,
            "root_ingress_bytes": sum(wire_sizes[1:]),
            "wire": fr.wire,
            "backend": args.backend,
            "note": "median of 5 frames whose steps run one after another, each timed alone after the timed "
                    "region: kernel_ms_per_rank = each rank's render kernel (11 synchronous launches), "
                    "pack = RGBA8 -> 3 B/px wire, gather = the transfer alone (all ranks packed before it "
                    "starts; HIP events around the RCCL gather, wall time of the host-staged gather with gloo), "
                    "deinterleave = rank 0's de-interleave kernel; the timed frames pipeline frame k's gather "
                    "and de-interleave with frame k+1's render",
        }
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
    elapsed, kern_max = float(t.item()), float(kt.item())

    if rank == 0:
        flop_rank = st["flop"]
        pmc = {}
        try:
            pm = json.load(open(args.pmc))
            # counters of one N = 1 launch of this frame at this pose (a rank's
            # share, or a walk's other poses, are priced per executed ray-step)
            pmc = pm.get(f"{args.scene}_{W}x{H}_{args.max_steps}_{args.pose}", {})
        except (OSError, ValueError):
            pass
        exact = world == 1 and not args.walk
        rank_launch[0]["kernel_ms"] = kern
        # the roofline's launch: the slowest rank's (kernel_ms_max_rank), priced
        # by its own executed ray-steps; every rank's beside it
        crit = max(range(len(rank_launch)), key=lambda q: rank_launch[q]["kernel_ms"])
        cl = rank_launch[crit]
        ms_step = elapsed / args.steps * 1e3
        # the roofline's launch duration: the median synchronous launch, never longer than the driver-timed step
        code_hash = rm.render_code_hash()
        roof = roofline(pmc, min(cl["kernel_ms"], ms_step), cl["executed_steps"],
                        W * cl["rows"] * (4 if args.fmt == "rgba8" else 16), flop_rank if crit == 0 else None,
                        evals_rank if crit == 0 else None, exact=exact, rows_frac=cl["rows"] / H, code_hash=code_hash)
        roof["render_code_hash"] = code_hash
        if world > 1:
            roof["rank"] = crit
            roof["per_rank_frac"] = [roofline(pmc, q["kernel_ms"], q["executed_steps"], 0, None, None, exact=False,
                                              rows_frac=q["rows"] / H, code_hash=code_hash)["frac"]
                                     for q in rank_launch]
        res = {
            "metric": "ray-steps/sec + frames/sec at 4096\u00d74096, 1/2/4/8 MI355X",
            "value": evals_frame * args.steps / elapsed,
            "unit": "ray-steps/s",
            "frames_per_s": args.steps / elapsed,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniforms only (camera pose), no input data",
            "config": {
                "workload": f"{_config_id(args.scene, W, H, args.max_steps, world)}: {W}x{H} scene {args.scene} "
                            f"({rm.SCENE_FILES[args.scene]}), {args.max_steps} max steps, pose {args.pose}, "
                            + (f"row bands of {args.band} over {world} GPU(s)" if fr.plan.runs is None else
                               f"weighted row runs {list(fr.plan.runs)} per cycle of {fr.plan.cycle} over "
                               f"{world} GPUs")
                            + (f", {fr.wire} wire" if world > 1 else "")
                            + f", {args.fmt} frame on rank 0"
                            + (f", walking (camera +{args.walk_speed}/frame forward, u_time +{args.walk_dt:.4f} s/frame)"
                               if args.walk else ""),
                "scene": args.scene, "W": W, "H": H, "max_steps": args.max_steps, "pose": args.pose,
                "band": args.band, "fmt": args.fmt, "wire": fr.wire, "streams": len(fr.streams), "kernel": args.kernel, "chunks": chunks, "schedule": args.schedule,
                "ray_steps_per_frame": evals_frame, "ray_steps_per_px": evals_frame / (W * H),
                "executed_ray_steps_per_frame": evals_frame - skipped_frame,
                "walk": None if not args.walk else {
                    "speed": args.walk_speed, "dt": args.walk_dt, "frames": args.steps,
                    "rank0_ray_steps_min": min(walk_evals), "rank0_ray_steps_max": max(walk_evals),
                    "end_pose": walk_pose(pose, args.steps - 1, args.walk_speed, args.walk_dt)},
            },
            "value_note": "value counts the reference's ray-steps (sceneSDF calls of common.frag's loops) per "
                          "frame; the kernels leave out steps that provably cannot change the frame (exact early "
                          "exits: settled soft shadows, the shadows of points facing away from the light, scene "
                          "T's reflection march past depth 3; DESIGN.md 2.11-2.13), so they execute "
                          "executed_ray_steps_per_s; frames_per_s is the same either way",
            "executed_ray_steps_per_s": (evals_frame - skipped_frame) * args.steps / elapsed,
            "kernel_ms": kern, "kernel_ms_max_rank": kern_max, "frame_stream_ms": frame_stream_ms,
            "kernel_ms_note": "median per-launch duration of the render kernel (HIP events on its stream, "
                              "synchronous launches after the timed region, adaptive dispatch order as in the "
                              "timed frames); frame_stream_ms = mean interval of the timed frames' render calls "
                              "(kernel + dispatch-order sort; with 2 streams it spans overlapping frames)",
            "roofline": roof,
            "frame_check": check,
        }
        if balance is not None:
            res["balance"] = balance
        if exchange is not None:
            res.update(exchange)
        if fr.frame is not None and fr.fmt == "rgba8":
            counters = load_post_counters(args.post_pmc)
            res["post_pass"] = time_fxaa(r, fr.frame, stream, counters)
            res["bloom_pass"] = time_bloom(r, fr.frame, stream, counters)
            if world == 1:
                res["pipeline"] = time_pipeline(r, W, H, stream, counters, res["ms_per_step"])
                res["pipeline_ms"] = res["pipeline"]["pipeline_ms"]
        if world == 1 and args.cpu_seconds > 0:
            res["cpu_baseline"] = cpu_baseline(args, pose, W, H, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
