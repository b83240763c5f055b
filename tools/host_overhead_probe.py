"""Host time per frame of the pipelined multi-GPU frame loops (DistributedFrame
over the RGB8 wire, DeltaFrame over the tile wire) with the GPU work made
negligible (a 64 x 64 frame): two ranks in one process, their collectives
replaced by device copies under the same stream semantics (as
tests/test_gpu_parity.py's in-process pipeline tests), each rank's submit()
timed on the host.  At N = 8 a rank's C3 share is ~0.075 ms of GPU time per
frame, so a loop whose host time per frame approaches that is host-bound.
One JSON line per loop.  (tools/; not product.)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import DeltaFrame, DistributedFrame  # noqa: E402

W, H, band, FRAMES = 64, 64, 8, 400
side = torch.cuda.Stream()


class Work:
    def __init__(self, entry=None, ev=None):
        self.entry, self.ev = entry, ev

    def wait(self):
        ev = self.ev if self.ev is not None else (self.entry or {}).get("done")
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)


def delta_pair():
    queue = []

    def fake(fr):
        def exchange(slot):
            if fr.rank == 1:
                fr.size_ev[slot].synchronize()
                mine = int(fr.size_host[slot][0])
                entry = {"msg": fr.msg[slot], "size": mine}
                queue.append(entry)
                return [0, mine], [Work(entry)]
            entry = queue.pop(0)
            if fr.decoded_recorded[slot]:
                side.wait_event(fr.decoded[slot])
            with torch.cuda.stream(side):
                fr.recv[slot][1][: entry["size"]].copy_(entry["msg"][: entry["size"]])
            done = torch.cuda.Event()
            done.record(side)
            entry["done"] = done
            return [0, entry["size"]], [Work(ev=done)]
        return exchange

    frs = []
    for rank in (0, 1):
        r = renderer()
        f = DeltaFrame.__new__(DeltaFrame)
        f._pipelined = lambda: True
        DeltaFrame.__init__(f, r, W, H, band, rank, 2)
        f._sizes_and_messages = fake(f)
        frs.append(f)
    return frs


class FakeWork:
    def __init__(self, ev=None):
        self.ev = ev

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)


def rgb8_pair():
    sent = {}

    def fake_gather(fr):
        def gather(slot, c):
            ev = torch.cuda.Event()
            ev.record()
            j0, j1 = 0, fr.plan.rows_per_shard
            if fr.rank == 1:
                sent[fr.k] = (fr.wires[slot][j0:j1], ev)
                return [FakeWork()]
            src1, ev1 = sent.pop(fr.k)
            side.wait_event(ev)
            side.wait_event(ev1)
            with torch.cuda.stream(side):
                fr.gathered[slot][0, j0:j1].copy_(fr.wires[slot][j0:j1])
                fr.gathered[slot][1, j0:j1].copy_(src1)
            done = torch.cuda.Event()
            done.record(side)
            return [FakeWork(done)]
        return gather

    frs = []
    for rank in (0, 1):
        r = renderer()
        f = DistributedFrame.__new__(DistributedFrame)
        f._pipelined = lambda: True
        DistributedFrame.__init__(f, r, W, H, band, rank, 2, fmt="rgba8")
        f._gather_async = fake_gather(f)
        frs.append(f)
    return frs


def renderer():
    r = rm.Renderer(0)
    r.load_scene(rm.SCENE_FILES["T"])
    r.set_uniform("u_resolution", W, H)
    p = rm.POSES["P0"]
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=16, count_evals=0)
    return r


def timed(frs):
    host = [0.0, 0.0]
    for i in range(20):
        frs[1].submit()
        frs[0].submit()
    torch.cuda.synchronize()
    for i in range(FRAMES):
        for q in (1, 0):
            t0 = time.perf_counter()
            frs[q].submit()
            host[q] += time.perf_counter() - t0
    frs[1].flush()
    frs[0].flush()
    torch.cuda.synchronize()
    return [h / FRAMES * 1e3 for h in host]


if os.environ.get("PROFILE"):  # cProfile of both ranks' submits (the hot host calls)
    import cProfile
    import pstats
    for make in (rgb8_pair, delta_pair):
        frs = make()
        pr = cProfile.Profile()
        pr.enable()
        timed(frs)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(22)
    sys.exit(0)
frs = rgb8_pair()
h = timed(frs)
print(json.dumps({"loop": "DistributedFrame (RGB8 wire), gather faked", "host_ms_per_frame": {"root": h[0],
                  "other": h[1]}, "frame": [W, H]}), flush=True)
frs = delta_pair()
h = timed(frs)
print(json.dumps({"loop": "DeltaFrame (tile wire), exchange faked", "host_ms_per_frame": {"root": h[0], "other": h[1]},
                  "frame": [W, H]}), flush=True)
