"""Host-side mirror of the reference's shader-pass surface, over librm.so.

The reference drives its ray-march pass through SFML (main.cpp:52-54,187-207):

    sf::Shader shader;
    ShaderLoader::loadFromFile("output_shader.frag", sf::Shader::Fragment, shader);
    shader.setUniform("u_resolution", sf::Vector2f(wf, hf));
    ...
    shader.setUniform("u_pos", pos); shader.setUniform("u_mouse", ...);
    shader.setUniform("u_time", t);
    outputTexture.draw(firstTextureSpriteFlipped, &shader);

The same names, argument meaning and error behaviour exist here:
``ShaderLoader.loadFromFile(file, Shader.Fragment, shader) -> bool`` (prints
and returns False on failure, source/shader_loader.cpp:26-30),
``Shader.setUniform(name, value)`` and ``RenderTexture.draw(shader)``, whose
target is a W x H x 4 float32 tensor resident in HBM.  ``Renderer`` is the
lower-level handle (one librm context) used by bench.py and the tests.
"""
from __future__ import annotations

import ctypes
import sys

from . import _lib
from ._lib import RmParams, RmStats, check, lib


def _torch():
    import torch  # noqa: PLC0415  (torch provides device memory and streams only)
    return torch


class Renderer:
    """One librm context on one HIP device."""

    def __init__(self, device: int = 0):
        L = lib()
        self._ctx = ctypes.c_void_p()
        st = L.rm_create(ctypes.byref(self._ctx), int(device))
        if st != 0:
            raise _lib.RmError(st, f"rm_create(device={device}) failed")
        self.device = int(device)

    def close(self):
        if self._ctx:
            lib().rm_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    # --- state ---------------------------------------------------------
    def load_scene(self, name: str) -> None:
        check(lib().rm_load_scene(self._ctx, name.encode()), self._ctx)

    def set_uniform(self, name: str, *v: float) -> None:
        L = lib()
        n = name.encode()
        if len(v) == 1:
            st = L.rm_set_uniform1f(self._ctx, n, float(v[0]))
        elif len(v) == 2:
            st = L.rm_set_uniform2f(self._ctx, n, float(v[0]), float(v[1]))
        elif len(v) == 3:
            st = L.rm_set_uniform3f(self._ctx, n, float(v[0]), float(v[1]), float(v[2]))
        else:
            raise ValueError("uniforms have 1..3 float components")
        check(st, self._ctx)

    def set_pose(self, pos, mouse, time) -> None:
        self.set_uniform("u_pos", *pos)
        self.set_uniform("u_mouse", *mouse)
        self.set_uniform("u_time", time)

    def set_params(self, max_steps=None, shadow_max_steps=None, count_evals=None, kernel=None,
                   schedule=None) -> None:
        p = self.params()
        if schedule is not None:
            p.schedule = {"adaptive": 1, "rowmajor": 0}.get(schedule, schedule)
        if max_steps is not None:
            p.max_steps = int(max_steps)
        if shadow_max_steps is not None:
            p.shadow_max_steps = int(shadow_max_steps)
        if count_evals is not None:
            p.count_evals = int(bool(count_evals))
        if kernel is not None:
            p.kernel = {"auto": 0, "tile16": 1, "tile8": 2, "tile16x4": 3, "persist": 4}.get(kernel, kernel)
        check(lib().rm_set_params(self._ctx, ctypes.byref(p)), self._ctx)

    def params(self) -> RmParams:
        p = RmParams()
        check(lib().rm_get_params(self._ctx, ctypes.byref(p)), self._ctx)
        return p

    def set_stream(self, stream, kept: bool = False) -> None:
        """stream: a torch.cuda.Stream, a raw hipStream_t int, or None.  kept:
        the stream outlives this renderer (rm_set_stream_kept; PyTorch's pool
        streams are never destroyed), so leaving it records no marker."""
        raw = getattr(stream, "cuda_stream", stream)
        fn = lib().rm_set_stream_kept if kept else lib().rm_set_stream
        check(fn(self._ctx, ctypes.c_void_p(raw or 0)), self._ctx)

    def tile_grid(self, W: int, rows: int) -> tuple:
        """(tiles_x, tiles_y) of a render launch over W x rows pixels."""
        tx, ty = ctypes.c_int(), ctypes.c_int()
        p = self.params()
        check(lib().rm_tile_grid(ctypes.byref(p), int(W), int(rows), ctypes.byref(tx), ctypes.byref(ty)))
        return tx.value, ty.value

    def set_tile_order(self, order=None) -> None:
        """rm_set_tile_order: workgroup i renders tile order[i] (None clears)."""
        import numpy as np
        if order is None:
            check(lib().rm_set_tile_order(self._ctx, None, 0), self._ctx)
            return
        o = np.ascontiguousarray(order, np.uint32)
        check(lib().rm_set_tile_order(self._ctx, ctypes.c_void_p(o.ctypes.data), len(o)), self._ctx)

    def synchronize(self) -> None:
        check(lib().rm_synchronize(self._ctx), self._ctx)

    # --- passes ----------------------------------------------------------
    @staticmethod
    def _ptr(t):
        return ctypes.c_void_p(t.data_ptr()) if hasattr(t, "data_ptr") else ctypes.c_void_p(t.ctypes.data)

    def render(self, W: int, H: int, out=None, stats: bool = False):
        """Full frame into `out` (device tensor [H,W,4] f32; allocated if None)."""
        torch = _torch()
        if out is None:
            out = torch.empty((H, W, 4), dtype=torch.float32, device=f"cuda:{self.device}")
        _check_out(out, H * W * 4)
        s = RmStats()
        check(lib().rm_render(self._ctx, int(W), int(H), self._ptr(out), ctypes.byref(s) if stats else None),
              self._ctx)
        return (out, s.as_dict()) if stats else out

    def render_accumulate(self, W: int, H: int, accum, stats: bool = False):
        """Progressive accumulation (rm_render_accumulate[_rgba8]): `accum` holds
        the previous frame (u_sample) and receives mix(u_sample, colour,
        u_sample_part), the colour rendered with the sub-pixel offset
        fract(u_seed1) - 0.5.  float32 [H, W, 4] or RGBA8 int32 [H, W] words."""
        torch = _torch()
        rgba8 = accum.dtype == torch.int32
        if not rgba8 and accum.dtype != torch.float32:
            raise ValueError("render_accumulate: accum must be float32 [H, W, 4] or int32 RGBA8 words [H, W]")
        _check_out(accum, H * W * (1 if rgba8 else 4))
        s = RmStats()
        fn = lib().rm_render_accumulate_rgba8 if rgba8 else lib().rm_render_accumulate
        check(fn(self._ctx, int(W), int(H), self._ptr(accum), ctypes.byref(s) if stats else None), self._ctx)
        return (accum, s.as_dict()) if stats else accum

    def render_step_map(self, W: int, H: int, out=None, evals_map=None):
        """Full frame plus the per-pixel sceneSDF call counts: (float32 [H, W, 4],
        int32 [H, W], stats), device tensors (allocated if None)."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        if out is None:
            out = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        if evals_map is None:
            evals_map = torch.empty((H, W), dtype=torch.int32, device=dev)
        _check_out(out, H * W * 4)
        _check_out(evals_map, H * W)
        s = RmStats()
        check(lib().rm_render_step_map(self._ctx, int(W), int(H), self._ptr(out), self._ptr(evals_map),
                                       ctypes.byref(s)), self._ctx)
        return out, evals_map, s.as_dict()

    def render_band(self, W: int, H: int, band: int, nshards: int, shard: int, out=None, stats: bool = False):
        """Rows y with (y // band) % nshards == shard, packed in increasing y."""
        torch = _torch()
        n = shard_rows(H, band, nshards, shard)
        if out is None:
            out = torch.empty((n, W, 4), dtype=torch.float32, device=f"cuda:{self.device}")
        _check_out(out, n * W * 4)
        s = RmStats()
        check(lib().rm_render_band(self._ctx, int(W), int(H), int(band), int(nshards), int(shard), self._ptr(out),
                                   ctypes.byref(s) if stats else None), self._ctx)
        return (out, s.as_dict()) if stats else out

    def render_rows(self, W, H, band, nshards, shard, row_begin, row_count, out, stats=False):
        """Packed rows [row_begin, row_begin + row_count) of a shard into `out`
        (float32 [rows, W, 4], or int32 [rows, W] RGBA8 words: the kernel packs)."""
        torch = _torch()
        rgba8 = out.dtype != torch.float32
        _check_out(out, row_count * W * (1 if rgba8 else 4))
        s = RmStats()
        fn = lib().rm_render_rows_rgba8 if rgba8 else lib().rm_render_rows
        check(fn(self._ctx, int(W), int(H), int(band), int(nshards), int(shard), int(row_begin), int(row_count),
                 self._ptr(out), ctypes.byref(s) if stats else None), self._ctx)
        return (out, s.as_dict()) if stats else out

    def render_cycle_rows(self, W, H, cycle, offset, run, row_begin, row_count, out, stats=False):
        """Packed rows [row_begin, row_begin + row_count) of the cyclic part
        (y mod cycle) - offset in [0, run), as render_rows (float32 or RGBA8 out)."""
        torch = _torch()
        rgba8 = out.dtype != torch.float32
        _check_out(out, row_count * W * (1 if rgba8 else 4))
        s = RmStats()
        fn = lib().rm_render_cycle_rows_rgba8 if rgba8 else lib().rm_render_cycle_rows
        check(fn(self._ctx, int(W), int(H), int(cycle), int(offset), int(run), int(row_begin), int(row_count),
                 self._ptr(out), ctypes.byref(s) if stats else None), self._ctx)
        return (out, s.as_dict()) if stats else out

    def deinterleave_cycle_rgb8(self, W, H, cycle, offsets, runs, part_bytes, gathered, out=None):
        """The RGBA8 frame (alpha 255) from cyclic parts' packed RGB8 rows:
        part i (offsets[i], runs[i], tiling [0, cycle) in order) starts at byte
        part_bytes[i] of the contiguous uint8 `gathered`."""
        torch = _torch()
        n = len(offsets)
        if len(runs) != n or len(part_bytes) != n:
            raise ValueError("deinterleave_cycle_rgb8: offsets, runs and part_bytes differ in length")
        if gathered.dtype != torch.uint8 or not gathered.is_contiguous():
            raise ValueError("deinterleave_cycle_rgb8: gathered must be a contiguous uint8 tensor")
        for o, r, b in zip(offsets, runs, part_bytes):
            if b + cycle_rows(H, cycle, o, r) * 3 * W > gathered.numel():
                raise ValueError("deinterleave_cycle_rgb8: a part's rows run past the end of gathered")
        if out is None:
            out = torch.empty((H, W), dtype=torch.int32, device=gathered.device)
        _check_out(out, H * W)
        check(lib().rm_deinterleave_cycle_rgb8(self._ctx, int(W), int(H), int(cycle), n,
                                               (ctypes.c_int * n)(*offsets), (ctypes.c_int * n)(*runs),
                                               (ctypes.c_int64 * n)(*part_bytes), self._ptr(gathered),
                                               self._ptr(out)), self._ctx)
        return out

    def render_cycle_rows_wire(self, W, H, cycle, offset, run, row_begin, row_count, msg, workspace, size_out=None,
                               stats=False):
        """render_cycle_rows's RGBA8 rows as the compressed wire's message,
        encoded by the render kernel's epilogue (rm_render_cycle_rows_wire):
        `msg` uint8 of wire_capacity(W, row_count) bytes, `workspace` of
        wire_workspace_bytes(W, row_count), `size_out` an optional int64
        device tensor [1] for the message size (asynchronously)."""
        torch = _torch()
        if msg.dtype != torch.uint8 or msg.numel() < wire_capacity(W, row_count) or not msg.is_contiguous():
            raise ValueError("render_cycle_rows_wire: msg must be a contiguous uint8 tensor of wire_capacity bytes")
        if workspace.numel() * workspace.element_size() < wire_workspace_bytes(W, row_count):
            raise ValueError("render_cycle_rows_wire: workspace too small")
        if size_out is not None and (size_out.dtype != torch.int64 or size_out.numel() < 1):
            raise ValueError("render_cycle_rows_wire: size_out must be an int64 tensor")
        s = RmStats()
        check(lib().rm_render_cycle_rows_wire(self._ctx, int(W), int(H), int(cycle), int(offset), int(run),
                                              int(row_begin), int(row_count), self._ptr(msg), self._ptr(workspace),
                                              self._ptr(size_out) if size_out is not None else None,
                                              ctypes.byref(s) if stats else None), self._ctx)
        return (msg, s.as_dict()) if stats else msg

    def wire_encode(self, rows, msg, workspace, size_out=None):
        """Compressed wire of packed RGBA8 rows (int32 [n, W]) into the uint8
        `msg` (>= wire_capacity bytes), with a uint8 `workspace` of
        wire_workspace_bytes; size_out: optional int64 device tensor [1] that
        receives the message size (asynchronously)."""
        torch = _torch()
        n, W = (int(rows.shape[0]), int(rows.shape[1])) if rows.dim() == 2 else (0, 0)
        if rows.dtype != torch.int32 or not rows.is_contiguous() or rows.dim() != 2:
            raise ValueError("wire_encode: rows must be contiguous int32 [n, W] RGBA8 words")
        if msg.dtype != torch.uint8 or msg.numel() < wire_capacity(W, n) or not msg.is_contiguous():
            raise ValueError("wire_encode: msg must be a contiguous uint8 tensor of wire_capacity bytes")
        if workspace.numel() * workspace.element_size() < wire_workspace_bytes(W, n):
            raise ValueError("wire_encode: workspace too small")
        if size_out is not None and (size_out.dtype != torch.int64 or size_out.numel() < 1):
            raise ValueError("wire_encode: size_out must be an int64 tensor")
        check(lib().rm_wire_encode(self._ctx, W, n, self._ptr(rows), self._ptr(msg), self._ptr(workspace),
                                   self._ptr(size_out) if size_out is not None else None), self._ctx)
        return msg

    def wire_decode(self, W, H, cycle, offset, run, nrows, msg, frame):
        """A wire message of `nrows` rows of the cyclic part into the int32
        [H, W] RGBA8 frame (alpha 255)."""
        _check_out(frame, H * W)
        check(lib().rm_wire_decode(self._ctx, int(W), int(H), int(cycle), int(offset), int(run), int(nrows),
                                   self._ptr(msg), self._ptr(frame)), self._ctx)
        return frame

    def wire_decode_parts(self, W, H, cycle, offsets, runs, nrows, msgs, frame):
        """rm_wire_decode_parts: several parts' messages (uint8 device tensors)
        into the int32 [H, W] frame in one launch."""
        _check_out(frame, H * W)
        n = len(msgs)
        check(lib().rm_wire_decode_parts(self._ctx, int(W), int(H), int(cycle), n, (ctypes.c_int * n)(*offsets),
                                         (ctypes.c_int * n)(*runs), (ctypes.c_int * n)(*nrows),
                                         (ctypes.c_void_p * n)(*[m.data_ptr() for m in msgs]), self._ptr(frame)),
              self._ctx)
        return frame

    def scatter_part_rgba8(self, W, H, cycle, offset, run, nrows, rows, frame):
        """A part's packed RGBA8 rows (int32 [nrows, W]) into their frame rows."""
        _check_out(frame, H * W)
        _check_out(rows, nrows * W)
        check(lib().rm_scatter_part_rgba8(self._ctx, int(W), int(H), int(cycle), int(offset), int(run), int(nrows),
                                          self._ptr(rows), self._ptr(frame)), self._ctx)
        return frame

    def render_band_rgba8(self, W, H, band, nshards, shard, out=None, stats=False):
        """render_band into RGBA8 words ([rows, W] int32)."""
        torch = _torch()
        n = shard_rows(H, band, nshards, shard)
        if out is None:
            out = torch.empty((n, W), dtype=torch.int32, device=f"cuda:{self.device}")
        _check_out(out, n * W)
        s = RmStats()
        check(lib().rm_render_band_rgba8(self._ctx, int(W), int(H), int(band), int(nshards), int(shard),
                                         self._ptr(out), ctypes.byref(s) if stats else None), self._ctx)
        return (out, s.as_dict()) if stats else out

    def deinterleave(self, W, H, band, nshards, rows_per_shard, gathered, out=None):
        """gathered: [nshards, rows_per_shard, W, 4] f32, [nshards, rows_per_shard, W] RGBA8 words, or
        [nshards, rows_per_shard, 3 * W] uint8 (the RGB8 wire; the frame is RGBA8 words, alpha 255)."""
        torch = _torch()
        if gathered.dtype == torch.uint8:
            if out is None:
                out = torch.empty((H, W), dtype=torch.int32, device=gathered.device)
            _check_out(out, H * W)
            if gathered.numel() < nshards * rows_per_shard * W * 3 or not gathered.is_contiguous():
                raise ValueError("deinterleave: RGB8 wire must be contiguous with 3*W bytes per row")
            check(lib().rm_deinterleave_rgb8(self._ctx, W, H, band, nshards, rows_per_shard, self._ptr(gathered),
                                             self._ptr(out)), self._ctx)
            return out
        rgba8 = gathered.dtype != torch.float32  # RGBA8 words travel as int32
        per_px = 1 if rgba8 else 4
        if out is None:
            shape = (H, W) if rgba8 else (H, W, 4)
            out = torch.empty(shape, dtype=gathered.dtype, device=gathered.device)
        _check_out(out, H * W * per_px)
        _check_out(gathered, nshards * rows_per_shard * W * per_px)
        fn = lib().rm_deinterleave_rgba8 if rgba8 else lib().rm_deinterleave
        check(fn(self._ctx, W, H, band, nshards, rows_per_shard, self._ptr(gathered), self._ptr(out)), self._ctx)
        return out

    def pack_rgb8(self, frame8, out=None):
        """RGBA8 words -> the 3 B/px RGB8 wire (alpha dropped; the pass writes alpha 1)."""
        torch = _torch()
        _check_out(frame8, frame8.numel())
        npx = frame8.numel()
        if out is None:
            out = torch.empty(tuple(frame8.shape[:-1]) + (3 * frame8.shape[-1],), dtype=torch.uint8,
                              device=frame8.device)
        if out.numel() < 3 * npx or out.dtype != torch.uint8 or not out.is_contiguous() or not frame8.is_contiguous():
            raise ValueError("pack_rgb8: out must be a contiguous uint8 tensor with 3 bytes per pixel")
        check(lib().rm_pack_rgb8(self._ctx, npx, self._ptr(frame8), self._ptr(out)), self._ctx)
        return out

    def pack_rgba8(self, frame, out=None):
        torch = _torch()
        if frame.dtype != torch.float32 or not frame.is_contiguous() or frame.numel() % 4:
            raise ValueError("pack_rgba8: frame must be a contiguous float32 tensor of RGBA pixels")
        npx = frame.numel() // 4
        if out is None:
            out = torch.empty(frame.shape[:-1], dtype=torch.int32, device=frame.device)
        if out.numel() < npx or out.element_size() != 4 or not out.is_contiguous():
            raise ValueError("pack_rgba8: out must be a contiguous 32-bit tensor with one element per pixel")
        check(lib().rm_pack_rgba8(self._ctx, npx, self._ptr(frame), self._ptr(out)), self._ctx)
        return out

    def fxaa(self, frame8, out=None):
        """post.frag's FXAA over an [H, W] RGBA8 (int32 words) device frame."""
        torch = _torch()
        H, W = frame8.shape
        if out is None:
            out = torch.empty_like(frame8)
        _check_out(frame8, H * W)
        _check_out(out, H * W)
        check(lib().rm_fxaa(self._ctx, W, H, self._ptr(frame8), self._ptr(out)), self._ctx)
        return out

    def bloom(self, frame8, out=None):
        """bloom.frag (with its mip chain) over an [H, W] RGBA8 (int32 words) device frame."""
        torch = _torch()
        H, W = frame8.shape
        if out is None:
            out = torch.empty_like(frame8)
        _check_out(frame8, H * W)
        _check_out(out, H * W)
        check(lib().rm_bloom(self._ctx, W, H, self._ptr(frame8), self._ptr(out)), self._ctx)
        return out

    def post_chain(self, frame8, mid=None, out=None):
        """main.cpp:209-214's post passes of a frame: FXAA of frame8 into mid,
        then bloom of mid into out (rm_post_chain); returns (mid, out)."""
        torch = _torch()
        H, W = frame8.shape
        if mid is None:
            mid = torch.empty_like(frame8)
        if out is None:
            out = torch.empty_like(frame8)
        for t in (frame8, mid, out):
            _check_out(t, H * W)
        check(lib().rm_post_chain(self._ctx, W, H, self._ptr(frame8), self._ptr(mid), self._ptr(out)), self._ctx)
        return mid, out

    def scene_eval(self, points, material: bool = False):
        """sceneSDF(p) of the loaded scene at points [n, 3] (host, numpy):
        dist [n], and with material=True also the [n, 16] Material floats."""
        import numpy as np
        pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        n = len(pts)
        dist = np.zeros(n, np.float32)
        mat = np.zeros((n, 16), np.float32) if material else None
        check(lib().rm_scene_eval(self._ctx, self._ptr(pts), n, self._ptr(dist),
                                  self._ptr(mat) if material else None), self._ctx)
        return (dist, mat) if material else dist

    def render_rgba8(self, W, H, out=None, stats=False):
        torch = _torch()
        if out is None:
            out = torch.empty((H, W), dtype=torch.int32, device=f"cuda:{self.device}")
        _check_out(out, H * W)
        s = RmStats()
        check(lib().rm_render_rgba8(self._ctx, W, H, self._ptr(out), ctypes.byref(s) if stats else None),
              self._ctx)
        return (out, s.as_dict()) if stats else out


def sharded_layout(W: int, H: int, band: int, nranks: int, rank: int) -> dict:
    """rm_sharded_layout: the row/byte layout of rm_render_sharded (no GPU)."""
    L = _lib.RmShardLayout()
    check(lib().rm_sharded_layout(int(W), int(H), int(band), int(nranks), int(rank), ctypes.byref(L)))
    return dict(rows_mine=L.rows_mine, rows_per_shard=L.rows_per_shard, wire_bytes=L.wire_bytes,
                gathered_bytes=L.gathered_bytes)


def comm_get_id() -> bytes:
    """rm_comm_get_id (ncclGetUniqueId): rank 0 makes it, every rank passes it to Comm."""
    cid = _lib.RmCommId()
    check(lib().rm_comm_get_id(ctypes.byref(cid)))
    return ctypes.string_at(ctypes.addressof(cid), 128)


class Comm:
    """A librm RCCL communicator bound to a Renderer (rm_comm_*): row-sharded
    RGBA8 frames, rank r rendering the rows (y // band) % nranks == r and
    rank 0 receiving the frame (rm_render_sharded)."""

    def __init__(self, renderer: Renderer, nranks: int = 1, rank: int = 0, comm_id: bytes | None = None,
                 _handle=None):
        self.r, self.nranks, self.rank = renderer, int(nranks), int(rank)
        if _handle is not None:
            self._h = _handle
            return
        cid = _lib.RmCommId()
        if comm_id is None and self.nranks == 1:
            comm_id = comm_get_id()  # a one-rank communicator needs no exchange of the id
        if comm_id is not None:
            ctypes.memmove(ctypes.addressof(cid), comm_id, 128)
        self._h = ctypes.c_void_p()
        check(lib().rm_comm_init_rank(ctypes.byref(self._h), renderer._ctx, self.nranks, ctypes.byref(cid),
                                      self.rank), renderer._ctx)

    @staticmethod
    def init_all(renderers) -> list:
        """One process driving len(renderers) GPUs (rm_comm_init_all)."""
        n = len(renderers)
        hs = (ctypes.c_void_p * n)()
        ctxs = (ctypes.c_void_p * n)(*[r._ctx.value for r in renderers])
        check(lib().rm_comm_init_all(hs, ctxs, n), renderers[0]._ctx)
        return [Comm(r, n, i, _handle=ctypes.c_void_p(hs[i])) for i, r in enumerate(renderers)]

    def render(self, W: int, H: int, band: int = 16, frame=None, stats: bool = False, runs=None):
        """One sharded frame (collective over the ranks).  Rank 0 gets the
        [H, W] RGBA8 (int32 words) frame, the others None.  runs: weighted
        parts (rm_render_sharded_runs, one run per rank) instead of bands."""
        torch = _torch()
        if self.rank == 0 and frame is None:
            frame = torch.empty((H, W), dtype=torch.int32, device=f"cuda:{self.r.device}")
        if frame is not None:
            _check_out(frame, H * W)
        s = RmStats()
        fp = self.r._ptr(frame) if frame is not None else None
        sp = ctypes.byref(s) if stats else None
        if runs is not None:
            if len(runs) != self.nranks:
                raise ValueError(f"runs needs {self.nranks} entries")
            check(lib().rm_render_sharded_runs(self._h, int(W), int(H), (ctypes.c_int * len(runs))(*runs), fp, sp),
                  self.r._ctx)
        else:
            check(lib().rm_render_sharded(self._h, int(W), int(H), int(band), fp, sp), self.r._ctx)
        return (frame, s.as_dict()) if stats else frame

    @staticmethod
    def render_all(comms, W: int, H: int, band: int = 16, frame=None, stats: bool = False, runs=None):
        """rm_render_sharded_all (or, with runs, rm_render_sharded_runs_all)
        over the communicators of init_all."""
        torch = _torch()
        n = len(comms)
        if frame is None:
            frame = torch.empty((H, W), dtype=torch.int32, device=f"cuda:{comms[0].r.device}")
        _check_out(frame, H * W)
        hs = (ctypes.c_void_p * n)(*[c._h.value for c in comms])
        st = (RmStats * n)()
        if runs is not None:
            if len(runs) != n:
                raise ValueError(f"runs needs {n} entries")
            check(lib().rm_render_sharded_runs_all(hs, n, int(W), int(H), (ctypes.c_int * n)(*runs),
                                                   comms[0].r._ptr(frame), st if stats else None), comms[0].r._ctx)
        else:
            check(lib().rm_render_sharded_all(hs, n, int(W), int(H), int(band), comms[0].r._ptr(frame),
                                              st if stats else None), comms[0].r._ctx)
        return (frame, [x.as_dict() for x in st]) if stats else frame

    @property
    def uses_rccl(self) -> bool:
        n, r, u = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().rm_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(u)))
        return bool(u.value)

    def close(self):
        if self._h:
            lib().rm_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def compile_scene(file_name: str):
    """rm_compile_scene: compile a scene plugin with hiprtc, no GPU needed.
    Returns (ok, log); a missing file or #include raises RmError."""
    buf = ctypes.create_string_buffer(1 << 16)
    st = lib().rm_compile_scene(file_name.encode(), ctypes.cast(buf, ctypes.c_void_p), len(buf))
    log = buf.value.decode(errors="replace")
    if st == _lib.STATUS_CODES["RM_ERR_FILE"]:
        raise _lib.RmError(st, log)
    return st == 0, log


def _check_out(t, nfloats):
    """A buffer the C ABI reads or writes as 32-bit words: a contiguous torch
    tensor or numpy array of 4-byte elements with at least `nfloats` of them."""
    if hasattr(t, "is_contiguous"):
        ok, n, es = t.is_contiguous(), t.numel(), t.element_size()
    else:
        ok, n, es = bool(t.flags["C_CONTIGUOUS"]), t.size, t.itemsize
    if not ok or n < nfloats or es != 4:
        raise ValueError(f"buffer must be contiguous 32-bit with >= {nfloats} elements")


def render_code_hash() -> str:
    """The render kernels' code objects by content (rm_render_code_hash): the
    build a PMC counter set was taken with (bench.py)."""
    return lib().rm_render_code_hash().decode()


def wire_capacity(W: int, nrows: int) -> int:
    """Largest wire message of nrows rows of W pixels (rm_wire_capacity)."""
    v = int(lib().rm_wire_capacity(int(W), int(nrows)))
    if v < 0:
        raise ValueError("wire_capacity: bad size")
    return v


def wire_workspace_bytes(W: int, nrows: int) -> int:
    v = int(lib().rm_wire_workspace_bytes(int(W), int(nrows)))
    if v < 0:
        raise ValueError("wire_workspace_bytes: bad size")
    return v


def cycle_rows(H: int, cycle: int, offset: int, run: int) -> int:
    """Frame rows y < H with (y mod cycle) - offset in [0, run) (rm_cycle_rows)."""
    n = ctypes.c_int()
    check(lib().rm_cycle_rows(int(H), int(cycle), int(offset), int(run), ctypes.byref(n)))
    return n.value


def shard_rows(H: int, band: int, nshards: int, shard: int) -> int:
    n = ctypes.c_int()
    check(lib().rm_shard_rows(int(H), int(band), int(nshards), int(shard), ctypes.byref(n)))
    return n.value


# ------------------------------------------------ the reference's surface


class Shader(Renderer):
    """sf::Shader as main.cpp uses it: a loaded scene plus its uniforms."""

    Fragment = "Fragment"

    def __init__(self, device: int = 0):
        super().__init__(device)
        self.loaded = False

    def setUniform(self, name: str, value) -> None:  # noqa: N802 (SFML name)
        vals = tuple(value) if isinstance(value, (tuple, list)) else (value,)
        self.set_uniform(name, *vals)


class ShaderLoader:
    """source/shader_loader.h:8-15."""

    @staticmethod
    def loadFromFile(file_name: str, type_, out_shader: Shader) -> bool:  # noqa: N802
        if type_ != Shader.Fragment:
            print(f"ShaderLoader: only fragment passes exist here (got {type_})", file=sys.stderr)
            return False
        try:
            out_shader.load_scene(file_name)
        except _lib.RmError as e:
            print(str(e), file=sys.stderr)
            return False
        out_shader.loaded = True
        return True


class RenderTexture:
    """sf::RenderTexture stand-in: a W x H float4 target resident in HBM."""

    def __init__(self):
        self.texture = None

    def create(self, W: int, H: int, device: int = 0) -> bool:
        torch = _torch()
        self.W, self.H = int(W), int(H)
        self.texture = torch.zeros((H, W, 4), dtype=torch.float32, device=f"cuda:{device}")
        return True

    def draw(self, shader: Shader, stats: bool = False):
        """Run `shader`'s pass over the whole target (main.cpp:199,205)."""
        r = shader.render(self.W, self.H, out=self.texture, stats=stats)
        return r[1] if stats else None

    def getTexture(self):  # noqa: N802
        return self.texture
