#!/usr/bin/env python3
"""N-GPU frame model from one GPU: every rank's share of an
N-way row split rendered on this GPU as that rank would render it in the
pipelined bench (two HIP streams, RGBA8 kernel + RGB8 pack per frame, frames
back to back; no gather), the root's de-interleave of the whole frame, and
the wire bytes each rank sends.  The projected frame time at N is

    max( max over ranks of the rank's per-frame compute (+ de-interleave on the root),
         the largest non-root wire / the assumed per-link xGMI rate )

(each non-root rank's rows cross their own link, concurrently, while the next
frame renders).  The link rate is an assumption (--link-gbs), printed with
the result; the driver's 8-GPU run measures the real gather (bench.py
gather_ms).  Both the even split (bands of 16) and bench.py's balanced split
(balanced_runs, sized with the same link assumption) are modelled.

--wire delta models the compressed wire (DeltaFrame) instead:
every non-root rank renders straight into its message
(rm_render_cycle_rows_wire, the encode in the render kernel's epilogue, plus
the scan and compaction), the root renders its rows, copies them into the
frame and decodes the other parts' real messages (their last frame's, one
rm_wire_decode_parts launch) in the same two-stream frame loop, so the
decode overlaps the next frame's render as in DeltaFrame (the decode alone is
also timed, root_decode_ms); the link carries the messages.

Usage: scale_model.py [--config C3|C5] [--ns 1,2,4,8] [--frames 24] [--link-gbs 64] [--wire rgb8|delta]
One JSON line per (N, split)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {  # scene, W, H, max steps, pose
    "C3": ("T", 4096, 4096, 256, "P0"),
    "C5": ("O", 8192, 8192, 512, "P0"),
    "C3P1": ("T", 4096, 4096, 256, "P1"),
}


def cumask_stream(torch):
    """A HIP stream created with an all-CU mask: the runtime gives a CU-masked
    stream a hardware queue of its own instead of sharing the least-used one."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(st.value)


STREAM_KIND = "pool"
KEPT = False  # --kept: frame streams bound with rm_set_stream_kept, as DistributedFrame binds them
WIRE = "rgb8"


def per_frame_ms(r, torch, plan, rank, frames, nstreams=2):
    """Rank's pipelined per-frame compute: render (RGBA8) + pack (RGB8) on two
    alternating streams, `frames` frames, wall time / frames."""
    p = plan
    n = p.count(rank)
    if n == 0:
        return 0.0, 0.0
    W = p.W
    if STREAM_KIND == "cumask":
        streams = [cumask_stream(torch) for _ in range(nstreams)]
    elif STREAM_KIND == "probed" and nstreams > 1:  # as DistributedFrame picks them
        from raymarching_amd.frame import concurrent_streams
        streams = concurrent_streams(torch.device("cuda:0"), nstreams)
    else:
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    loc = [torch.empty((n, W), dtype=torch.int32, device="cuda") for _ in streams]
    wire = [torch.empty((n, 3 * W), dtype=torch.uint8, device="cuda") for _ in streams]
    delta = WIRE == "delta"
    if delta:
        import raymarching_amd as rm
        msg = [torch.empty(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda") for _ in streams]
        ws = [torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda") for _ in streams]
        size = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in streams]
        frame = torch.empty((p.H, W), dtype=torch.int32, device="cuda") if rank == 0 else None

    def one(i):
        k = i % nstreams
        st = streams[k]
        with torch.cuda.stream(st):
            r.set_stream(st, kept=KEPT)
            if not delta:
                r.render_cycle_rows(W, p.H, p.cycle, p.offsets[rank], p.part_runs[rank], 0, n, loc[k])
                r.pack_rgb8(loc[k], out=wire[k])
            elif rank == 0:  # its rows into the frame, then the other parts' messages decoded into it
                r.render_cycle_rows(W, p.H, p.cycle, p.offsets[rank], p.part_runs[rank], 0, n, loc[k])
                r.scatter_part_rgba8(W, p.H, p.cycle, p.offsets[rank], p.part_runs[rank], n, loc[k], frame)
                if len(MESSAGES) == p.nshards - 1:
                    qs = range(1, p.nshards)
                    r.wire_decode_parts(W, p.H, p.cycle, [p.offsets[q] for q in qs], [p.part_runs[q] for q in qs],
                                        [MESSAGES[q][1] for q in qs], [MESSAGES[q][0] for q in qs], frame)
            else:
                r.render_cycle_rows_wire(W, p.H, p.cycle, p.offsets[rank], p.part_runs[rank], 0, n, msg[k], ws[k],
                                         size[k])
        r.set_stream(streams[0], kept=KEPT)

    t_end = time.time() + 0.3
    i = 0
    while time.time() < t_end or i < 16:  # clock ramp + adaptive order settled on both streams
        one(i)
        i += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(frames):
        one(j)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / frames * 1e3
    # single synchronous launch (the bench's kernel_ms) for the record
    r.set_stream(streams[0])
    ks = sorted(r.render_cycle_rows(W, p.H, p.cycle, p.offsets[rank], p.part_runs[rank], 0, n, loc[0],
                                    stats=True)[1]["kernel_ms"] for _ in range(7))
    if delta and rank > 0:  # this rank's message (the last frame's), for the root's decode and the link
        torch.cuda.synchronize()
        k = int(size[0].item())
        MESSAGES[rank] = (msg[0][:k].clone(), n)
    return ms, ks[len(ks) // 2]


MESSAGES = {}  # rank -> (message, rows) of the last modelled plan (--wire delta)


def per_rank(r, torch, plan, args):
    """Every rank's per_frame_ms; with the compressed wire the other ranks
    first, so that the root's frames decode their messages."""
    order = list(range(1, plan.nshards)) + [0] if WIRE == "delta" else list(range(plan.nshards))
    out = {q: per_frame_ms(r, torch, plan, q, args.frames, args.streams) for q in order}
    return [out[q] for q in range(plan.nshards)]


def decode_ms(r, torch, plan):
    """The root's decode of every other part's message into the frame (one launch)."""
    W, H = plan.W, plan.H
    r.set_stream(torch.cuda.current_stream())  # (the frame loop left a frame stream bound: time on the events' one)
    frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
    qs = list(range(1, plan.nshards))
    args = (W, H, plan.cycle, [plan.offsets[q] for q in qs], [plan.part_runs[q] for q in qs],
            [MESSAGES[q][1] for q in qs], [MESSAGES[q][0] for q in qs], frame)
    for _ in range(10):
        r.wire_decode_parts(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        r.wire_decode_parts(*args)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 30


def deinterleave_ms(r, torch, plan):
    W, H = plan.W, plan.H
    r.set_stream(torch.cuda.current_stream())
    g = torch.randint(0, 255, (H, 3 * W), dtype=torch.uint8, device="cuda")
    out = torch.empty((H, W), dtype=torch.int32, device="cuda")
    bases = [b * 3 * W for b in plan.part_bases()]
    args = (W, H, plan.cycle, list(plan.offsets), list(plan.part_runs), bases, g)
    for _ in range(20):
        r.deinterleave_cycle_rgb8(*args, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        r.deinterleave_cycle_rgb8(*args, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 50


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--band", type=int, default=16)
    ap.add_argument("--streams", type=int, default=2, help="frames in flight per rank (HIP streams)")
    ap.add_argument("--even-only", action="store_true")
    ap.add_argument("--kept", action="store_true", help="bind the frame streams as kept (no marker per leave)")
    ap.add_argument("--stream-kind", default="probed", choices=["pool", "cumask", "probed"])
    ap.add_argument("--wire", default="rgb8", choices=["rgb8", "delta"])
    ap.add_argument("--link-gbs", type=float, default=64.0,
                    help="assumed xGMI rate of one link, one direction, as RCCL point-to-point achieves it (GB/s)")
    args = ap.parse_args()
    import torch
    global STREAM_KIND, KEPT, WIRE
    STREAM_KIND = args.stream_kind
    KEPT = args.kept
    WIRE = args.wire

    import raymarching_amd as rm
    from bench import balanced_runs
    from raymarching_amd.frame import ShardPlan

    scene, W, H, steps, pose = CONFIGS[args.config]
    r = rm.Renderer(0)
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    pz = rm.POSES[pose]
    r.set_pose(pz["pos"], pz["mouse"], pz["time"])
    r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=0, schedule=1)
    link_bpms = args.link_gbs * 1e6  # bytes per ms
    for N in [int(x) for x in args.ns.split(",")]:
        even = ShardPlan(W, H, args.band if N > 1 else H, N, None if N > 1 else (H,))
        MESSAGES.clear()
        per = per_rank(r, torch, even, args)
        d = (decode_ms(r, torch, even) if args.wire == "delta" else deinterleave_ms(r, torch, even)) if N > 1 else 0.0
        wire_even = ([0] + [int(MESSAGES[q][0].numel()) for q in range(1, N)] if args.wire == "delta" and N > 1
                     else None)
        rows = {"even": (even, per, d, wire_even)}
        if N > 1 and not args.even_only:
            # the root's run sized so that its rows plus the decode (or de-interleave)
            # take as long as another rank's rows or its link time (bench.balanced_runs)
            gbytes = max(wire_even[1:]) if wire_even else max(even.count(q) for q in range(1, N)) * 3 * W
            ex = {"render_ms": [x[0] for x in per], "gather_ms": gbytes / link_bpms, "deinterleave_ms": d}
            runs, model = balanced_runs(N, args.band, H, ex)
            if tuple(runs) != tuple(even.part_runs):
                bal = ShardPlan(W, H, args.band, N, tuple(runs))
                MESSAGES.clear()
                perb = per_rank(r, torch, bal, args)
                if args.wire == "delta":
                    rows["balanced"] = (bal, perb, decode_ms(r, torch, bal),
                                        [0] + [int(MESSAGES[q][0].numel()) for q in range(1, N)])
                else:
                    rows["balanced"] = (bal, perb, deinterleave_ms(r, torch, bal), None)
        for name, (plan, pr, dms, wire) in rows.items():
            wire = wire if wire is not None else [plan.count(q) * 3 * W for q in range(N)]
            link = max(wire[1:], default=0) / link_bpms
            # (with the compressed wire the root's frames already decode the others' messages)
            compute = [pr[0][0] + (dms if args.wire == "rgb8" else 0.0)] + [x[0] for x in pr[1:]]
            frame = max(max(compute), link)
            print(json.dumps({
                "config": args.config, "N": N, "split": name, "wire": args.wire, "streams": args.streams,
                "stream_kind": args.stream_kind, "runs": list(plan.part_runs),
                "per_rank_frame_ms": [round(x[0], 4) for x in pr],
                "per_rank_kernel_ms": [round(x[1], 4) for x in pr],
                ("root_decode_ms" if args.wire == "delta" else "deinterleave_ms"): round(dms, 4),
                "root_frame_includes_decode": args.wire == "delta", "wire_bytes": wire,
                "link_gbs_assumed": args.link_gbs,
                "link_ms": round(link, 4), "projected_frame_ms": round(frame, 4),
                "bound": "link" if link >= max(compute) else ("root" if compute[0] >= max(compute[1:], default=0)
                                                              else "rank"),
            }), flush=True)
    r.close()


if __name__ == "__main__":
    main()
