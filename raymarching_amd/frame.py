"""Row-sharded frames across GPUs (one process per GPU, RCCL over xGMI).

Pixels are independent, so a frame shards by rows.  Rows are dealt to ranks
in bands of ``band`` rows, round robin: rank r owns frame row y iff
``(y // band) % nshards == r`` (cheap sky rows and expensive sponge / floor
rows spread evenly).  Each rank renders its rows packed in
increasing y (``rm_render_rows``, or ``rm_render_rows_rgba8``, whose kernel
packs RGBA8 in its epilogue), and one gather brings every band to the root, where
``rm_deinterleave`` writes the frame.  The gather is the only collective on
the path (``torch.distributed.gather``; the "nccl" backend is RCCL).

``ShardPlan`` is pure layout logic and is shared with the CPU (gloo) tests.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ShardPlan:
    """Which frame rows each shard renders.  Every shard owns one run of
    consecutive rows in each cycle of ``cycle`` rows: shard s owns row y iff
    ``(y mod cycle) - offsets[s]`` lies in ``[0, runs[s])``.  ``runs`` None is
    round-robin bands (every run = ``band``); explicit ``runs`` weight the
    shards (bench.py's balanced split gives the root, which also receives
    every other shard's rows, a longer run)."""
    W: int
    H: int
    band: int
    nshards: int
    runs: tuple | None = None

    def __post_init__(self):
        if self.runs is not None and (len(self.runs) != self.nshards or min(self.runs) < 1):
            raise ValueError(f"runs must hold {self.nshards} positive row counts, got {self.runs}")

    @property
    def weighted(self) -> bool:
        return self.runs is not None

    @property
    def part_runs(self) -> tuple:
        return tuple(self.runs) if self.runs is not None else (self.band,) * self.nshards

    @property
    def cycle(self) -> int:
        return sum(self.part_runs)

    @property
    def offsets(self) -> tuple:
        o, acc = [], 0
        for r in self.part_runs:
            o.append(acc)
            acc += r
        return tuple(o)

    def rows(self, shard: int) -> list[int]:
        """Frame rows of `shard`, in packed (increasing) order."""
        c, o, r = self.cycle, self.offsets[shard], self.part_runs[shard]
        return [y for y in range(self.H) if 0 <= y % c - o < r]

    def count(self, shard: int) -> int:
        c, o, r = self.cycle, self.offsets[shard], self.part_runs[shard]
        full, rest = divmod(self.H, c)
        return full * r + min(max(rest - o, 0), r)

    @property
    def rows_per_shard(self) -> int:
        """Rows of the gather slot of every shard (the largest shard)."""
        return max(self.count(s) for s in range(self.nshards))

    def slot_of_row(self, y: int) -> tuple[int, int]:
        """(shard, packed row) holding frame row y."""
        cyc, m = divmod(y, self.cycle)
        offs, runs = self.offsets, self.part_runs
        s = max(i for i in range(self.nshards) if offs[i] <= m)
        return s, cyc * runs[s] + m - offs[s]

    def gathered_index(self):
        """Flat index into the [nshards * rows_per_shard] gathered rows for every frame row."""
        rps = self.rows_per_shard
        return [s * rps + j for s, j in (self.slot_of_row(y) for y in range(self.H))]

    def part_bases(self) -> list[int]:
        """First row of each shard in the unpadded gather (shards back to back)."""
        b, acc = [], 0
        for s in range(self.nshards):
            b.append(acc)
            acc += self.count(s)
        return b

    def packed_index(self):
        """Flat index into the unpadded gathered rows for every frame row."""
        base = self.part_bases()
        return [base[s] + j for s, j in (self.slot_of_row(y) for y in range(self.H))]


def gather_to_root(local, plan: ShardPlan, rank: int, group=None, out=None):
    """Gather each rank's packed rows (padded to rows_per_shard) into a
    [nshards, rows_per_shard, ...] tensor on rank 0 (None elsewhere).

    With the "nccl" backend (RCCL on ROCm) device buffers go over xGMI
    directly.  The "gloo" backend (CPU tests, and single-GPU rehearsals of the
    multi-rank path) moves host memory, so device buffers are staged.
    """
    import torch
    import torch.distributed as dist

    rps = plan.rows_per_shard
    if local.shape[0] != rps:
        raise ValueError(f"local band buffer must have rows_per_shard={rps} rows, has {local.shape[0]}")
    staged = local.is_cuda and dist.get_backend(group) == "gloo"
    src = local.cpu() if staged else local
    if rank == 0:
        if out is None:
            out = torch.empty((plan.nshards,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        dst = torch.empty(out.shape, dtype=out.dtype) if staged else out
        dist.gather(src, gather_list=list(dst.unbind(0)), dst=0, group=group)
        if staged:
            out.copy_(dst)
        return out
    dist.gather(src, gather_list=None, dst=0, group=group)
    return None


def gather_parts_to_root(local, plan: ShardPlan, rank: int, group=None, out=None):
    """Gather each rank's packed rows, unpadded, into the [sum of counts, ...]
    tensor `out` on rank 0 (shards back to back, ShardPlan.part_bases), with
    point-to-point sends: the shards of a weighted plan differ in size.  Rank
    0's own rows must already be in place (its render writes there).  gloo
    (host memory) stages device buffers; the CPU tests use it."""
    import torch
    import torch.distributed as dist

    staged = local.is_cuda and dist.get_backend(group) == "gloo"
    if rank == 0:
        base = plan.part_bases()
        for r in range(1, plan.nshards):
            n = plan.count(r)
            if n == 0:
                continue
            dst = out[base[r]: base[r] + n]
            buf = torch.empty(dst.shape, dtype=dst.dtype) if staged else dst
            dist.recv(buf, src=r, group=group)
            if staged:
                dst.copy_(buf)
        return out
    n = plan.count(rank)
    if local.shape[0] < n:
        raise ValueError(f"local rows {local.shape[0]} < this shard's {n}")
    if n:
        dist.send(local[:n].cpu() if staged else local[:n].contiguous(), dst=0, group=group)
    return None


def _runs_concurrently(a, b, cycles=400_000):
    """True if kernels on streams a and b overlap: a spin kernel on each, the
    pair timed on the host.  Two streams that share a hardware queue run one
    after the other."""
    import time

    import torch
    spin = getattr(torch.cuda, "_sleep", None)
    if spin is None:
        return True
    best = float("inf"), float("inf")
    for _ in range(2):
        ts = []
        for streams in ((a,), (a, b)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for st in streams:
                with torch.cuda.stream(st):
                    spin(cycles)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        best = min(best[0], ts[0]), min(best[1], ts[1])
    return best[1] < 1.5 * best[0]


def concurrent_streams(dev, n, tries=12):
    """n HIP streams of `dev` whose kernels run concurrently.  HIP maps a
    process's streams onto at most GPU_MAX_HW_QUEUES hardware queues (4 on
    MI355X nodes by default) and two streams on one queue serialize; which
    streams share depends on how many the process (PyTorch's pool, RCCL) made
    before, so the pairs are probed (tools/queue_probe.py: 1 in 4 to 1 in 8
    pool streams shared a queue with the default stream).  Falls back to the
    last candidates if none of `tries` qualify."""
    import torch
    with torch.cuda.device(dev):
        chosen = [torch.cuda.Stream(dev)]
        for _ in range(tries):
            if len(chosen) == n:
                break
            c = torch.cuda.Stream(dev)
            if all(_runs_concurrently(c, s) for s in chosen):
                chosen.append(c)
        while len(chosen) < n:
            chosen.append(torch.cuda.Stream(dev))
    return chosen


class _OnStream:
    """`with torch.cuda.stream(st)` for a stream of a known device, without the
    current-device queries of torch's StreamContext (a frame at N = 8 is
    ~0.08 ms of GPU time: the multi-GPU loops' host time per frame has to stay
    below that; tools/host_overhead_probe.py)."""
    __slots__ = ("st", "prev")

    def __init__(self, st):
        self.st = st

    def __enter__(self):
        import torch
        self.prev = torch.cuda.current_stream(self.st.device)
        torch.cuda.set_stream(self.st)
        return self.st

    def __exit__(self, *exc):
        import torch
        torch.cuda.set_stream(self.prev)
        return False


class DistributedFrame:
    """One rank's share of a row-sharded frame on its GPU.

    ``render()`` runs this rank's rows, gathers to rank 0 and (on rank 0)
    de-interleaves the frame; everything is asynchronous on the frame's
    stream.  ``fmt`` is "rgba8" (the displayed RenderTexture format; 3 B/px on
    the wire, ``wire="rgb8"``, or 4 with ``wire="rgba8"``) or "float4" (full
    gl_FragColor, 16 B/px, used by parity tests).

    Overlap, three ways:
    * ``submit()`` / ``flush()`` pipeline consecutive frames: frame k's gather
      runs on RCCL's stream while frame k+1 renders (the wire buffers are
      double-buffered); rank 0 de-interleaves frame k after frame k+1's render
      was enqueued.  One render launch per frame per rank.
    * ``streams=2`` puts consecutive frames on two HIP streams, so frame k+1's
      waves fill the SIMDs while frame k's longest waves finish.  A frame's
      time is bounded below by its slowest pixel (a grazing soft-shadow march
      of several hundred dependent steps); with 1/8 of a 4096^2 frame per rank
      that tail is as long as the rest of the frame, and overlapping frames
      hides it (tools/shard_probe.py: 0.23 -> 0.12 ms per rank at N = 8).
      Every buffer a frame writes (band, wire, gathered, frame) is per slot.
      Default: 2 streams when N > 1 and the gather is pipelined (RCCL), else 1.
    * ``chunks`` > 1 pipelines within a frame: the packed rows are cut into
      that many ranges (same cuts on every rank) and chunk k+1 renders while
      chunk k is gathered; it costs a launch tail per chunk.
    """

    def __init__(self, renderer, W, H, band, rank, world, fmt="rgba8", group=None, chunks=1, wire="auto",
                 streams=None, runs=None):
        import torch

        self.r, self.rank, self.world, self.fmt, self.group = renderer, rank, world, fmt, group
        # RGBA8 frames cross the wire as RGB8 (3 B/px: alpha is 1 by construction,
        # rm_pack_rgb8); the root restores alpha while de-interleaving.
        if wire == "auto":
            wire = "rgb8" if fmt == "rgba8" and world > 1 else fmt
        if wire not in (fmt, "rgb8") or (wire == "rgb8" and fmt != "rgba8"):
            raise ValueError(f"wire {wire!r} does not carry {fmt!r} frames")
        self.wire = wire
        # one shard: the packed rows are the frame rows (no de-interleave needed)
        if runs is not None and world > 1:
            # weighted parts: unpadded point-to-point gather of RGB8 rows
            if wire != "rgb8":
                raise ValueError("weighted row parts (runs) need the RGB8 wire (fmt='rgba8')")
            self.plan = ShardPlan(W, H, band, world, tuple(int(x) for x in runs))
        else:
            self.plan = ShardPlan(W, H, band if world > 1 else H, world)
        dev = torch.device(f"cuda:{renderer.device}")
        if streams is None:
            streams = 2 if self._pipelined() else 1
        if streams not in (1, 2):
            raise ValueError("streams must be 1 or 2")
        # one stream: the caller's; two: a probed pair that does not share a
        # hardware queue (on one queue the frames would not overlap)
        self.caller = torch.cuda.current_stream(dev)
        self.streams = [self.caller] if streams == 1 else concurrent_streams(dev, streams)
        if streams > 1:  # the frame streams start after the caller's work so far
            for st in self.streams:
                st.wait_stream(self.caller)
        rps = self.plan.rows_per_shard
        self.nmine = self.plan.count(rank)
        chunks = max(1, min(int(chunks), rps))
        if self.plan.weighted:
            # every shard cuts its own rows into the same number of chunks
            self.all_cuts = [[round(c * self.plan.count(q) / chunks) for c in range(chunks + 1)]
                             for q in range(world)]
            self.cuts = self.all_cuts[rank]
        else:
            self.cuts = [round(c * rps / chunks) for c in range(chunks + 1)]
        nbuf = 2 if world > 1 or streams > 1 else 1
        shape = (rps, W) if fmt == "rgba8" else (rps, W, 4)
        dtype = torch.int32 if fmt == "rgba8" else torch.float32
        if self.plan.weighted:
            # shards back to back in the root's gather buffer; the root packs its
            # own rows straight into the head of it
            n = self.nmine
            self.locals = [torch.empty((n, W), dtype=dtype, device=dev) for _ in range(nbuf)]
            if rank == 0:
                self.gathered = [torch.empty((H, 3 * W), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
                self.wires = [g[:n] for g in self.gathered]
            else:
                self.gathered = None
                self.wires = [torch.empty((n, 3 * W), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        elif self.wire == "rgb8":
            # render into a local RGBA8 band, pack each chunk into the slot being gathered
            self.locals = [torch.empty(shape, dtype=dtype, device=dev) for _ in range(nbuf)]
            self.wires = [torch.empty((rps, 3 * W), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        else:
            # the render kernel writes straight into the slot being gathered
            self.locals = None
            self.wires = [torch.empty(shape, dtype=dtype, device=dev) for _ in range(nbuf)]
        if not self.plan.weighted:
            wire = self.wires[0]
            self.gathered = ([torch.empty((world,) + tuple(wire.shape), dtype=wire.dtype, device=dev)
                              for _ in range(2)] if rank == 0 and world > 1 else None)
        if world == 1:
            self.frames = self.wires if self.locals is None else self.locals
        elif rank == 0:
            self.frames = [torch.empty((H, W) if fmt == "rgba8" else (H, W, 4), dtype=dtype, device=dev)
                           for _ in range(2)]
        else:
            self.frames = None
        self.frame = self.frames[0] if self.frames is not None else None
        self.k = 0            # frames submitted
        self.pending = None   # (slot, stream, [works]) of the frame whose gather is in flight
        self._pipe = self._pipelined()
        self._prepare_calls()

    def _prepare_calls(self):
        """The per-frame native calls of submit() with their arguments built
        once per slot and chunk (render, RGB8 pack, the root's de-interleave):
        the Python wrappers' checks cost as much host time as a rank's frame
        takes on the GPU at N = 8."""
        import ctypes

        import torch

        from ._lib import lib
        L, p, ctx = lib(), self.plan, self.r._ctx
        rgba8 = self.fmt == "rgba8"

        def vp(t):
            return ctypes.c_void_p(t.data_ptr())

        self._render_calls, self._pack_calls, self._deint_calls = [], [], []
        for slot in range(len(self.wires)):
            dst = self.wires[slot] if self.locals is None else self.locals[slot]
            rc, pc = [], []
            for c in range(len(self.cuts) - 1):
                j0, j1 = self.cuts[c], min(self.cuts[c + 1], self.nmine)
                if j1 <= j0:
                    rc.append(None)
                    pc.append(None)
                    continue
                if p.weighted:
                    fn = L.rm_render_cycle_rows_rgba8 if rgba8 else L.rm_render_cycle_rows
                    args = (ctx, p.W, p.H, p.cycle, p.offsets[self.rank], p.part_runs[self.rank], j0, j1 - j0,
                            vp(dst[j0:j1]), None)
                else:
                    fn = L.rm_render_rows_rgba8 if rgba8 else L.rm_render_rows
                    args = (ctx, p.W, p.H, p.band, p.nshards, self.rank, j0, j1 - j0, vp(dst[j0:j1]), None)
                rc.append((fn, args))
                pc.append((L.rm_pack_rgb8, (ctx, (j1 - j0) * p.W, vp(self.locals[slot][j0:j1]),
                                            vp(self.wires[slot][j0:j1]))) if self.locals is not None else None)
            self._render_calls.append(rc)
            self._pack_calls.append(pc)
            d = None
            if self.rank == 0 and self.world > 1 and self.gathered is not None:
                g, f = self.gathered[slot], self.frames[slot]
                if p.weighted:
                    n = p.nshards
                    d = (L.rm_deinterleave_cycle_rgb8,
                         (ctx, p.W, p.H, p.cycle, n, (ctypes.c_int * n)(*p.offsets), (ctypes.c_int * n)(*p.part_runs),
                          (ctypes.c_int64 * n)(*[b * 3 * p.W for b in p.part_bases()]), vp(g), vp(f)))
                elif g.dtype == torch.uint8:
                    d = (L.rm_deinterleave_rgb8, (ctx, p.W, p.H, p.band, p.nshards, p.rows_per_shard, vp(g), vp(f)))
                else:
                    fn = L.rm_deinterleave_rgba8 if rgba8 else L.rm_deinterleave
                    d = (fn, (ctx, p.W, p.H, p.band, p.nshards, p.rows_per_shard, vp(g), vp(f)))
            self._deint_calls.append(d)

    def _native(self, call):
        from ._lib import check
        rc = call[0](*call[1])
        if rc:
            check(rc, self.r._ctx)

    def _pipelined(self):
        import torch.distributed as dist
        return self.world > 1 and dist.get_backend(self.group) != "gloo"

    def _render_into(self, dst, j0, j1, stats=False):
        """Packed rows [j0, j1) of this rank's part into dst[j0:j1]."""
        p = self.plan
        if p.weighted:
            return self.r.render_cycle_rows(p.W, p.H, p.cycle, p.offsets[self.rank], p.part_runs[self.rank], j0,
                                            j1 - j0, dst[j0:j1], stats=stats)
        return self.r.render_rows(p.W, p.H, p.band, p.nshards, self.rank, j0, j1 - j0, dst[j0:j1], stats=stats)

    def _render_rows(self, c, slot, events=None, st=None):
        """Chunk c of this rank's rows into slot `slot` (and packed to RGB8), on
        the current stream st."""
        call = self._render_calls[slot][c]
        if call is None:
            return
        if events is not None:
            events[0].record(st)
        self._native(call)
        if events is not None:
            events[1].record(st)
        if self._pack_calls[slot][c] is not None:
            self._native(self._pack_calls[slot][c])

    def _gather_views(self, slot, c):
        """The tensors of chunk c's gather (c None: every row), cached per slot
        and chunk (slicing them per frame costs host time at N = 8): for
        point-to-point parts the (peer, tensor) pairs, else (send, gather_list)."""
        key = (slot, c)
        cache = self.__dict__.setdefault("_views", {})
        if key in cache:
            return cache[key]
        p = self.plan
        if p.weighted:
            pairs = []
            if self.rank == 0:
                base = p.part_bases()
                for q in range(1, self.world):
                    cq = self.all_cuts[q]
                    j0, j1 = (0, p.count(q)) if c is None else (cq[c], cq[c + 1])
                    if j1 > j0:
                        pairs.append((q, self.gathered[slot][base[q] + j0: base[q] + j1]))
            else:
                j0, j1 = (0, self.nmine) if c is None else (self.cuts[c], self.cuts[c + 1])
                if j1 > j0:
                    pairs.append((0, self.wires[slot][j0:j1]))
            v = pairs
        else:
            j0, j1 = (0, p.rows_per_shard) if c is None else (self.cuts[c], self.cuts[c + 1])
            g = self.gathered[slot] if self.rank == 0 else None
            v = (self.wires[slot][j0:j1], [g[r, j0:j1] for r in range(self.world)] if self.rank == 0 else None)
        cache[key] = v
        return v

    def _gather_async(self, slot, c):
        """Start chunk c's gather (c None: every row); returns the works."""
        import torch.distributed as dist
        p = self.plan
        v = self._gather_views(slot, c)
        if p.weighted:  # point-to-point: the parts differ in size (the ops reused frame after frame)
            ops = self._views.get(("ops", slot, c))
            if ops is None:
                op = dist.irecv if self.rank == 0 else dist.isend
                ops = self._views[("ops", slot, c)] = [dist.P2POp(op, t, q, group=self.group) for q, t in v]
            return dist.batch_isend_irecv(ops) if ops else []
        return [dist.gather(v[0], gather_list=v[1], dst=0, group=self.group, async_op=True)]

    def _gather_blocking(self, slot):
        """The host-staged gather (gloo), completed inside the call."""
        if self.plan.weighted:
            gather_parts_to_root(self.wires[slot], self.plan, self.rank, group=self.group,
                                 out=self.gathered[slot] if self.rank == 0 else None)
        else:
            gather_to_root(self.wires[slot], self.plan, self.rank, group=self.group,
                           out=self.gathered[slot] if self.rank == 0 else None)

    def _deinterleave(self, slot):
        p = self.plan
        if p.weighted:
            self.r.deinterleave_cycle_rgb8(p.W, p.H, p.cycle, list(p.offsets), list(p.part_runs),
                                           [b * 3 * p.W for b in p.part_bases()], self.gathered[slot],
                                           out=self.frames[slot])
        else:
            self.r.deinterleave(p.W, p.H, p.band, p.nshards, p.rows_per_shard, self.gathered[slot],
                                out=self.frames[slot])

    def _bind(self, st):
        """Bind the renderer to frame stream st.  The frame streams other than
        the caller's come from PyTorch's pool, which never destroys them, so
        they are bound as kept (rm_set_stream_kept): leaving one records no
        marker."""
        self.r.set_stream(st, kept=st is not self.caller)

    def render_local(self, stats=False):
        """This rank's rows only, into slot 0 (no gather), on the first frame
        stream (whose adaptive tile order the frames use); stats: one
        synchronous launch.  Ordered before later work on the caller's stream."""
        import torch
        dst = self.wires[0] if self.locals is None else self.locals[0]
        st = self.streams[0]
        with torch.cuda.stream(st):
            self._bind(st)
            try:
                res = self._render_into(dst, 0, self.nmine, stats=stats)
            finally:
                self.r.set_stream(self.caller)
        if st is not self.caller:
            self.caller.wait_stream(st)
        return res

    def submit(self, events=None):
        """Enqueue one frame.  With N > 1 its gather stays in flight until the
        next submit()/flush().  events: optional list of (start, end)
        torch.cuda.Event pairs, one per chunk, recorded around the renders."""
        import torch

        slot = self.k % len(self.wires)
        st = self.streams[self.k % len(self.streams)]
        self.k += 1
        nch = len(self.cuts) - 1
        works = []
        with _OnStream(st):  # the collectives order themselves after this stream
            self._bind(st)
            for c in range(nch):
                self._render_rows(c, slot, None if events is None else events[c], st)
                if self._pipe:
                    works.extend(self._gather_async(slot, c))
            if self.world > 1 and not self._pipe:  # gloo: one host-staged gather, completed here
                self._gather_blocking(slot)
                works = None
        self.r.set_stream(self.caller)
        if self.world == 1:
            self.frame = self.frames[slot]
        prev, self.pending = self.pending, (slot, st, works) if self.world > 1 else None
        if prev is not None:
            self._complete(prev)
        return self.frame

    def _complete(self, item):
        import torch

        slot, st, works = item
        with _OnStream(st):
            self._bind(st)
            for w in works or ():
                w.wait()  # st waits for the gather
            if self.rank == 0:
                self._native(self._deint_calls[slot])
                self.frame = self.frames[slot]
        self.r.set_stream(self.caller)

    def flush(self):
        """Finish the frame in flight (rank 0: its de-interleaved frame is in
        .frame, ordered before later work on the caller's stream)."""
        import torch

        if self.pending is not None:
            item, self.pending = self.pending, None
            self._complete(item)
        for st in self.streams[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            self.streams[0].wait_event(ev)
        if self.streams[0] is not self.caller:  # ... and the caller's stream after them
            self.caller.wait_stream(self.streams[0])
        return self.frame

    def render(self, events=None):
        """One complete frame (submit + flush)."""
        self.submit(events)
        return self.flush()

    def timed_exchange(self):
        """(see _timed_exchange); the renderer is back on the caller's stream after it."""
        try:
            return self._timed_exchange()
        finally:
            self.r.set_stream(self.caller)

    def _timed_exchange(self):
        """One frame with its steps run one after another and each timed alone
        (nothing pipelined): this rank's render, the RGB8 pack, then -- once
        every rank has packed (barrier) -- the gather, and on rank 0 the
        de-interleave.  Collective (every rank calls it).  Returns ms per step:
        render_ms, pack_ms, gather_ms (the transfer alone: HIP events around the
        RCCL gather on the frame stream; with gloo, wall time of the host-staged
        gather), deinterleave_ms (rank 0, else 0).  The frame lands in slot 0."""
        import time

        import torch
        import torch.distributed as dist

        st, slot = self.streams[0], 0
        dev = torch.device(f"cuda:{self.r.device}")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        self.flush()
        torch.cuda.synchronize(dev)
        self._bind(st)
        with torch.cuda.stream(st):
            ev[0].record(st)
            if self.nmine:
                self._render_into(self.wires[slot] if self.locals is None else self.locals[slot], 0, self.nmine)
            ev[1].record(st)
            if self.locals is not None and self.nmine:
                self.r.pack_rgb8(self.locals[slot][: self.nmine], out=self.wires[slot][: self.nmine])
            ev[2].record(st)
        torch.cuda.synchronize(dev)
        out = dict(render_ms=ev[0].elapsed_time(ev[1]), pack_ms=ev[1].elapsed_time(ev[2]), gather_ms=0.0,
                   deinterleave_ms=0.0)
        if self.world == 1:
            return out
        dist.barrier(group=self.group)
        if self._pipelined():
            with torch.cuda.stream(st):
                ev[3].record(st)
                for w in self._gather_async(slot, None):
                    w.wait()  # st waits for the gather
                ev[4].record(st)
            torch.cuda.synchronize(dev)
            out["gather_ms"] = ev[3].elapsed_time(ev[4])
        else:  # gloo: host-staged, completes inside the call
            t0 = time.perf_counter()
            self._gather_blocking(slot)
            torch.cuda.synchronize(dev)
            out["gather_ms"] = (time.perf_counter() - t0) * 1e3
        if self.rank == 0:
            with torch.cuda.stream(st):
                ev[4].record(st)
                self._deinterleave(slot)
                ev[5].record(st)
            torch.cuda.synchronize(dev)
            out["deinterleave_ms"] = ev[4].elapsed_time(ev[5])
            self.frame = self.frames[slot]
        return out


class DeltaFrame(DistributedFrame):
    """A row-sharded RGBA8 frame whose parts cross the wire compressed
    (rm_wire_encode: a lossless delta code per 64-pixel row segment, 4-5x
    fewer bytes than RGB8 on rendered frames).  Same plans
    (bands or weighted runs), streams and pipelining as DistributedFrame.

    The messages differ in size from frame to frame and RCCL's point-to-point
    calls take their sizes on the host, so each frame has a size exchange:
    a rank's encoder writes its message size to the device, a pinned copy
    follows on the frame's stream, and when frame k is completed (during
    submit(k + 1), while frame k + 1 renders) the host reads it, the ranks
    all-gather the sizes on a control stream, and the unpadded messages move
    point to point.  Rank 0 copies its own rows into the frame
    (rm_scatter_part_rgba8) and decodes the others' messages straight into
    their frame rows (rm_wire_decode); no de-interleave pass."""

    def __init__(self, renderer, W, H, band, rank, world, group=None, chunks=1, streams=None, runs=None):
        import torch

        if world < 2:
            raise ValueError("DeltaFrame needs two or more ranks")
        if chunks != 1:
            raise ValueError("DeltaFrame sends whole parts (chunks=1)")
        self.r, self.rank, self.world, self.fmt, self.group = renderer, rank, world, "rgba8", group
        self.wire = "delta"
        self.plan = ShardPlan(W, H, band, world, None if runs is None else tuple(int(x) for x in runs))
        dev = torch.device(f"cuda:{renderer.device}")
        self.dev = dev
        if streams is None:
            streams = 2 if self._pipelined() else 1
        if streams not in (1, 2):
            raise ValueError("streams must be 1 or 2")
        self.caller = torch.cuda.current_stream(dev)
        self.streams = [self.caller] if streams == 1 else concurrent_streams(dev, streams)
        if streams > 1:
            for st in self.streams:
                st.wait_stream(self.caller)
        self.ctrl = torch.cuda.Stream(dev)
        from .api import wire_capacity, wire_workspace_bytes
        p = self.plan
        self.nmine = p.count(rank)
        self.cuts = [0, self.nmine]
        nbuf = 2
        self.locals = [torch.empty((self.nmine, W), dtype=torch.int32, device=dev) for _ in range(nbuf)]
        self.wires = self.locals  # (slot count; the bench reads wires[0] for the row width)
        if rank == 0:
            self.frames = [torch.empty((H, W), dtype=torch.int32, device=dev) for _ in range(nbuf)]
            self.recv = [{q: torch.empty(wire_capacity(W, p.count(q)), dtype=torch.uint8, device=dev)
                          for q in range(1, world)} for _ in range(nbuf)]
            self.decoded = [torch.cuda.Event() for _ in range(nbuf)]
            self.decoded_recorded = [False] * nbuf
        else:
            self.frames = None
            self.msg = [torch.empty(wire_capacity(W, self.nmine), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
            self.ws = [torch.empty(wire_workspace_bytes(W, self.nmine), dtype=torch.uint8, device=dev)
                       for _ in range(nbuf)]
            self.size_dev = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(nbuf)]
            self.size_host = [torch.zeros(1, dtype=torch.int64).pin_memory() for _ in range(nbuf)]
            self.size_ev = [torch.cuda.Event() for _ in range(nbuf)]
        self.slot_works = [[] for _ in range(nbuf)]
        self.frame = self.frames[0] if self.frames is not None else None
        self.k = 0
        self.pending = None
        self.last_sizes = [0] * world
        self.fused = rank != 0  # (the render kernel encodes; scene plugins fall back, _render_message)
        self._pipe = self._pipelined()
        self._zero_size = torch.zeros(1, dtype=torch.int64, device=dev)
        self._allsz = [torch.zeros(world, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        # the per-frame native calls with their arguments built once (a frame
        # at N = 8 is ~0.1 ms: Python-side argument checks per call would cost
        # as much as the GPU work)
        import ctypes

        from ._lib import lib
        self._L = lib()
        if rank == 0:
            # the root's own rows (as _render_into, its arguments built once)
            vp = ctypes.c_void_p
            if p.weighted:
                self._root_render = [(self._L.rm_render_cycle_rows_rgba8,
                                      (renderer._ctx, W, H, p.cycle, p.offsets[0], p.part_runs[0], 0, self.nmine,
                                       vp(t.data_ptr()), None)) for t in self.locals]
            else:
                self._root_render = [(self._L.rm_render_rows_rgba8,
                                      (renderer._ctx, W, H, p.band, p.nshards, 0, 0, self.nmine, vp(t.data_ptr()),
                                       None)) for t in self.locals]
            qs = list(range(1, world))
            self._dec = [((ctypes.c_int * len(qs))(*[p.offsets[q] for q in qs]),
                          (ctypes.c_int * len(qs))(*[p.part_runs[q] for q in qs]),
                          (ctypes.c_int * len(qs))(*[p.count(q) for q in qs]),
                          (ctypes.c_void_p * len(qs))(*[self.recv[s_][q].data_ptr() for q in qs]))
                         for s_ in range(nbuf)]

    def _call(self, rc):
        from ._lib import check
        check(rc, self.r._ctx)

    def _encode(self, slot):
        self._call(self._L.rm_wire_encode(self.r._ctx, self.plan.W, self.nmine, self.locals[slot].data_ptr(),
                                          self.msg[slot].data_ptr(), self.ws[slot].data_ptr(),
                                          self.size_dev[slot].data_ptr()))

    def _render_message(self, slot, stats=False):
        """A non-root rank's part straight into its message: the render
        kernel encodes its tiles in its epilogue (rm_render_cycle_rows_wire);
        a scene plugin's part is rendered to rows and encoded after."""
        import ctypes

        from ._lib import RmError, RmStats
        p, q = self.plan, self.rank
        if self.fused:
            s = RmStats() if stats else None
            try:
                self._call(self._L.rm_render_cycle_rows_wire(
                    self.r._ctx, p.W, p.H, p.cycle, p.offsets[q], p.part_runs[q], 0, self.nmine,
                    self.msg[slot].data_ptr(), self.ws[slot].data_ptr(), self.size_dev[slot].data_ptr(),
                    ctypes.byref(s) if stats else None))
                return s.as_dict() if stats else None
            except RmError as e:
                if "built-in scenes only" not in str(e):
                    raise
                self.fused = False  # (a scene plugin: the two calls below from now on)
        st = None
        if self.nmine:
            st = self._render_into(self.locals[slot], 0, self.nmine, stats=stats)
        self._encode(slot)
        return st[1] if stats and st is not None else None

    def _scatter(self, slot):
        p = self.plan
        self._call(self._L.rm_scatter_part_rgba8(self.r._ctx, p.W, p.H, p.cycle, p.offsets[0], p.part_runs[0],
                                                 self.nmine, self.locals[slot].data_ptr(),
                                                 self.frames[slot].data_ptr()))

    def _produce(self, slot, st, events=None):
        """Render this rank's rows into slot `slot` on stream st, then (root)
        copy them into the frame or (others) encode them."""
        import torch
        p = self.plan
        with _OnStream(st):
            self._bind(st)
            for w in self.slot_works[slot]:  # the slot's previous message has left
                w.wait()
            self.slot_works[slot] = []
            if events is not None:
                events[0].record()
            if self.rank == 0:
                if self.nmine:
                    self._call(self._root_render[slot][0](*self._root_render[slot][1]))
                if events is not None:
                    events[1].record()
                self._scatter(slot)
            else:
                self._render_message(slot)  # (render and encode: one kernel plus the scan and compaction)
                if events is not None:
                    events[1].record()
                self.size_host[slot].copy_(self.size_dev[slot], non_blocking=True)
                self.size_ev[slot].record(st)
        self.r.set_stream(self.caller)

    def _sizes_and_messages(self, slot):
        """The size exchange of the frame in `slot`, then its messages posted
        (RCCL: on the control stream, returning the works; gloo: host-staged,
        completed).  Returns (sizes, works).  Collective."""
        import torch
        import torch.distributed as dist
        if self.rank == 0:
            mine = 0
        else:
            self.size_ev[slot].synchronize()  # the encoder's size has reached the host
            mine = int(self.size_host[slot][0])
        if self._pipe:
            with _OnStream(self.ctrl):
                # (the encoder's device size, complete once size_ev was reached;
                # preallocated buffers: no allocation or fill per frame)
                src = self.size_dev[slot] if self.rank else self._zero_size
                dist.all_gather_into_tensor(self._allsz[slot], src, group=self.group)
                sizes = self._allsz[slot].tolist()
                self._check_sizes(sizes)  # (every rank: all fail together, before any send or receive)
                if self.rank == 0:
                    if self.decoded_recorded[slot]:
                        self.ctrl.wait_event(self.decoded[slot])  # the slot's last decode has read its buffers
                    ops = [dist.P2POp(dist.irecv, self.recv[slot][q][: sizes[q]], q, group=self.group)
                           for q in range(1, self.world)]
                else:
                    ops = [dist.P2POp(dist.isend, self.msg[slot][:mine], 0, group=self.group)]
                return sizes, dist.batch_isend_irecv(ops)
        allsz = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        dist.all_gather(allsz, torch.tensor([mine], dtype=torch.int64), group=self.group)
        sizes = [int(v[0]) for v in allsz]
        self._check_sizes(sizes)  # (every rank: all fail together, before any send or receive)
        if self.rank == 0:
            for q in range(1, self.world):
                buf = torch.empty(sizes[q], dtype=torch.uint8)
                dist.recv(buf, src=q, group=self.group)
                self.recv[slot][q][: sizes[q]].copy_(buf)
        else:
            dist.send(self.msg[slot][:mine].cpu(), dst=0, group=self.group)
        return sizes, []

    def _check_sizes(self, sizes):
        """The ranks' message sizes against the wire capacity of their parts
        (rank 0's receive buffers): a larger one would be truncated and the
        send/receive lengths would no longer match (a hang or a corrupt
        decode), so it fails here instead -- on every rank, which all hold
        the gathered sizes, so no peer is left blocked in a send until the
        process group's timeout."""
        from .api import wire_capacity
        for q in range(1, self.world):
            cap = wire_capacity(self.plan.W, self.plan.count(q))
            if not 0 <= sizes[q] <= cap:
                raise RuntimeError(f"DeltaFrame: rank {q} reports a {sizes[q]}-byte message; the receive buffer "
                                   f"holds {cap} (wire capacity)")

    def _decode(self, slot, st):
        p = self.plan
        self._call(self._L.rm_wire_decode_parts(self.r._ctx, p.W, p.H, p.cycle, self.world - 1, *self._dec[slot],
                                                self.frames[slot].data_ptr()))

    def _exchange(self, slot, st):
        """Sizes, messages, and on rank 0 the decodes into its frame on st."""
        import torch
        sizes, works = self._sizes_and_messages(slot)
        self.last_sizes = sizes
        if self.rank == 0:
            with _OnStream(st):
                self._bind(st)
                for w in works:
                    w.wait()
                self._decode(slot, st)
                self.decoded[slot].record(st)
                self.decoded_recorded[slot] = True
            self.r.set_stream(self.caller)
            self.frame = self.frames[slot]
        else:
            self.slot_works[slot] = works

    def submit(self, events=None):
        slot = self.k % 2
        st = self.streams[self.k % len(self.streams)]
        self.k += 1
        self._produce(slot, st, None if events is None else events[0])
        prev, self.pending = self.pending, (slot, st)
        if not self._pipe:
            self.pending = None
            self._exchange(slot, st)
        elif prev is not None:
            self._exchange(*prev)
        return self.frame

    def flush(self):
        import torch
        if self.pending is not None:
            item, self.pending = self.pending, None
            self._exchange(*item)
        for st in self.streams[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            self.streams[0].wait_event(ev)
        if self.streams[0] is not self.caller:
            self.caller.wait_stream(self.streams[0])
        for ws in self.slot_works:  # the caller's stream after every message has left
            for w in ws:
                w.wait()
        return self.frame

    def render_local(self, stats=False):
        """This rank's part once (rank 0: its rows; the others: their message,
        as the frames make it); with stats, (rows or message, rm_stats)."""
        import torch
        st = self.streams[0]
        with torch.cuda.stream(st):
            self._bind(st)
            try:
                if self.rank == 0:
                    res = self._render_into(self.locals[0], 0, self.nmine, stats=stats)
                else:
                    s = self._render_message(0, stats=stats)
                    res = (self.msg[0], s) if stats else self.msg[0]
            finally:
                self.r.set_stream(self.caller)
        if st is not self.caller:
            self.caller.wait_stream(st)
        return res

    def timed_exchange(self):
        """render_ms (this rank's rows), pack_ms (encode, or the root's copy
        into the frame), gather_ms (wall: size exchange + messages), and on
        rank 0 deinterleave_ms (the decodes, events); wire_bytes: the sizes."""
        import time

        import torch
        import torch.distributed as dist
        self.flush()
        torch.cuda.synchronize(self.dev)
        st, slot = self.streams[0], 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        p = self.plan
        with torch.cuda.stream(st):
            self._bind(st)
            ev[0].record(st)
            if self.rank == 0:
                if self.nmine:
                    self._render_into(self.locals[slot], 0, self.nmine)
                ev[1].record(st)
                self._scatter(slot)
            else:
                # render + encode in one kernel (the scan and compaction after it count as the pack)
                self._render_message(slot)
                ev[1].record(st)
                self.size_host[slot].copy_(self.size_dev[slot], non_blocking=True)
                self.size_ev[slot].record(st)
            ev[2].record(st)
        self.r.set_stream(self.caller)
        torch.cuda.synchronize(self.dev)
        out = dict(render_ms=ev[0].elapsed_time(ev[1]), pack_ms=ev[1].elapsed_time(ev[2]))
        dist.barrier(group=self.group)
        t0 = time.perf_counter()
        sizes, works = self._sizes_and_messages(slot)
        for w in works:
            w.wait()
        torch.cuda.synchronize(self.dev)
        out["gather_ms"] = (time.perf_counter() - t0) * 1e3
        out["deinterleave_ms"] = 0.0
        if self.rank == 0:
            with torch.cuda.stream(st):
                self._bind(st)
                ev[3].record(st)
                self._decode(slot, st)
                ev[4].record(st)
                self.decoded[slot].record(st)
                self.decoded_recorded[slot] = True
            self.r.set_stream(self.caller)
            torch.cuda.synchronize(self.dev)
            out["deinterleave_ms"] = ev[3].elapsed_time(ev[4])
            self.frame = self.frames[slot]
        out["wire_bytes"] = sizes
        return out
