"""ctypes binding of librm.so (include/rm.h).

The product path has no CPU fallback: if librm.so is missing or fails to
load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RM_LIB may point at an alternative in-tree build (experiments); default librm.so
LIB_PATH = os.environ.get("RM_LIB") or os.path.join(HERE, "librm.so")

RM_OK = 0
STATUS = {0: "RM_OK", 1: "RM_ERR_INVALID_ARGUMENT", 2: "RM_ERR_FILE", 3: "RM_ERR_SCENE",
          4: "RM_ERR_NO_SCENE", 5: "RM_ERR_DEVICE", 6: "RM_ERR_OUT_OF_MEMORY"}
STATUS_CODES = {v: k for k, v in STATUS.items()}

# every symbol include/rm.h declares
EXPORTS = ("rm_create", "rm_destroy", "rm_load_scene", "rm_set_uniform1f", "rm_set_uniform2f",
           "rm_set_uniform3f", "rm_set_params", "rm_get_params", "rm_set_stream", "rm_set_stream_kept",
           "rm_synchronize",
           "rm_render", "rm_render_band", "rm_render_rows", "rm_shard_rows", "rm_deinterleave", "rm_deinterleave_rgba8",
           "rm_pack_rgba8", "rm_pack_rgb8", "rm_deinterleave_rgb8",
           "rm_render_rgba8", "rm_render_accumulate", "rm_render_accumulate_rgba8", "rm_render_band_rgba8", "rm_render_rows_rgba8", "rm_fxaa", "rm_bloom", "rm_post_chain", "rm_render_code_hash", "rm_render_cycle_rows_wire", "rm_last_error", "rm_status_string",
           "rm_compile_scene", "rm_scene_eval", "rm_render_step_map", "rm_sharded_layout", "rm_comm_get_id",
           "rm_comm_init_rank", "rm_comm_init_all", "rm_comm_destroy", "rm_render_sharded", "rm_render_sharded_all",
           "rm_set_tile_order", "rm_tile_grid", "rm_comm_info", "rm_abi_version", "rm_cycle_rows",
           "rm_render_cycle_rows", "rm_render_cycle_rows_rgba8", "rm_deinterleave_cycle_rgb8",
           "rm_render_sharded_runs", "rm_render_sharded_runs_all", "rm_wire_capacity", "rm_wire_workspace_bytes",
           "rm_wire_encode", "rm_wire_decode", "rm_scatter_part_rgba8", "rm_wire_decode_parts")

# include/rm.h RM_ABI_VERSION: the struct layouts below
ABI_VERSION = 3
DISPATCH = {0: "row-major", 1: "explicit", 2: "adaptive"}


class RmParams(ctypes.Structure):
    _fields_ = [("max_steps", ctypes.c_int32), ("shadow_max_steps", ctypes.c_int32),
                ("count_evals", ctypes.c_int32), ("kernel", ctypes.c_int32), ("schedule", ctypes.c_int32)]


class RmStats(ctypes.Structure):
    _fields_ = [("evals", ctypes.c_uint64), ("pixels", ctypes.c_uint64), ("kernel_ms", ctypes.c_float),
                ("scene", ctypes.c_int32), ("flop", ctypes.c_uint64), ("skipped", ctypes.c_uint64),
                ("dispatch", ctypes.c_int32), ("lat_tiles", ctypes.c_int32), ("gather_ms", ctypes.c_float),
                ("deinterleave_ms", ctypes.c_float)]

    def as_dict(self):
        return dict(evals=int(self.evals), pixels=int(self.pixels), kernel_ms=float(self.kernel_ms),
                    scene=int(self.scene), flop=int(self.flop), skipped=int(self.skipped),
                    dispatch=DISPATCH.get(int(self.dispatch), int(self.dispatch)), lat_tiles=int(self.lat_tiles),
                    gather_ms=float(self.gather_ms), deinterleave_ms=float(self.deinterleave_ms))


class RmShardLayout(ctypes.Structure):
    _fields_ = [("rows_mine", ctypes.c_int32), ("rows_per_shard", ctypes.c_int32), ("wire_bytes", ctypes.c_int64),
                ("gathered_bytes", ctypes.c_int64)]


class RmCommId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class RmError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


_LIB = None


def lib() -> ctypes.CDLL:
    """Load librm.so (raises if it is missing: no fallback path exists)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run `make -C raymarching_amd` (or __graft_entry__.build())")
    # torch ships its own libamdhip64.so.7: load it first so that librm.so binds
    # to the same HIP runtime (one runtime per process; tensors and streams
    # are then shared).  A process without torch uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401,PLC0415
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, c = ctypes.c_void_p, ctypes
    cp = c.c_char_p
    sig = {
        "rm_create": ([c.POINTER(vp), c.c_int], c.c_int),
        "rm_destroy": ([vp], c.c_int),
        "rm_load_scene": ([vp, cp], c.c_int),
        "rm_set_uniform1f": ([vp, cp, c.c_float], c.c_int),
        "rm_set_uniform2f": ([vp, cp, c.c_float, c.c_float], c.c_int),
        "rm_set_uniform3f": ([vp, cp, c.c_float, c.c_float, c.c_float], c.c_int),
        "rm_set_params": ([vp, c.POINTER(RmParams)], c.c_int),
        "rm_get_params": ([vp, c.POINTER(RmParams)], c.c_int),
        "rm_set_stream": ([vp, vp], c.c_int),
        "rm_set_stream_kept": ([vp, vp], c.c_int),
        "rm_synchronize": ([vp], c.c_int),
        "rm_render": ([vp, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_step_map": ([vp, c.c_int, c.c_int, vp, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_band": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_rows": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp,
                            c.POINTER(RmStats)], c.c_int),
        "rm_shard_rows": ([c.c_int, c.c_int, c.c_int, c.c_int, c.POINTER(c.c_int)], c.c_int),
        "rm_deinterleave": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_deinterleave_rgba8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_pack_rgba8": ([vp, c.c_int64, vp, vp], c.c_int),
        "rm_pack_rgb8": ([vp, c.c_int64, vp, vp], c.c_int),
        "rm_deinterleave_rgb8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_render_rgba8": ([vp, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_accumulate": ([vp, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_accumulate_rgba8": ([vp, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_band_rgba8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, c.POINTER(RmStats)],
                                 c.c_int),
        "rm_render_rows_rgba8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp,
                                  c.POINTER(RmStats)], c.c_int),
        "rm_fxaa": ([vp, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_bloom": ([vp, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_post_chain": ([vp, c.c_int, c.c_int, vp, vp, vp], c.c_int),
        "rm_render_code_hash": ([], cp),
        "rm_render_cycle_rows_wire": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp, vp,
                                       c.POINTER(RmStats)], c.c_int),
        "rm_compile_scene": ([cp, vp, c.c_size_t], c.c_int),
        "rm_scene_eval": ([vp, vp, c.c_int64, vp, vp], c.c_int),
        "rm_sharded_layout": ([c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.POINTER(RmShardLayout)], c.c_int),
        "rm_comm_get_id": ([c.POINTER(RmCommId)], c.c_int),
        "rm_comm_init_rank": ([c.POINTER(vp), vp, c.c_int, c.POINTER(RmCommId), c.c_int], c.c_int),
        "rm_comm_init_all": ([c.POINTER(vp), c.POINTER(vp), c.c_int], c.c_int),
        "rm_comm_destroy": ([vp], c.c_int),
        "rm_comm_info": ([vp, c.POINTER(c.c_int), c.POINTER(c.c_int), c.POINTER(c.c_int)], c.c_int),
        "rm_render_sharded": ([vp, c.c_int, c.c_int, c.c_int, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_sharded_all": ([c.POINTER(vp), c.c_int, c.c_int, c.c_int, c.c_int, vp, c.POINTER(RmStats)],
                                  c.c_int),
        "rm_set_tile_order": ([vp, vp, c.c_int64], c.c_int),
        "rm_tile_grid": ([c.POINTER(RmParams), c.c_int, c.c_int, c.POINTER(c.c_int), c.POINTER(c.c_int)], c.c_int),
        "rm_abi_version": ([], c.c_int),
        "rm_cycle_rows": ([c.c_int, c.c_int, c.c_int, c.c_int, c.POINTER(c.c_int)], c.c_int),
        "rm_render_cycle_rows": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp,
                                  c.POINTER(RmStats)], c.c_int),
        "rm_render_cycle_rows_rgba8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp,
                                        c.POINTER(RmStats)], c.c_int),
        "rm_deinterleave_cycle_rgb8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp, vp, vp, vp], c.c_int),
        "rm_wire_capacity": ([c.c_int, c.c_int], c.c_int64),
        "rm_wire_workspace_bytes": ([c.c_int, c.c_int], c.c_int64),
        "rm_wire_encode": ([vp, c.c_int, c.c_int, vp, vp, vp, vp], c.c_int),
        "rm_wire_decode": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_scatter_part_rgba8": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp], c.c_int),
        "rm_wire_decode_parts": ([vp, c.c_int, c.c_int, c.c_int, c.c_int, vp, vp, vp, vp, vp], c.c_int),
        "rm_render_sharded_runs": ([vp, c.c_int, c.c_int, vp, vp, c.POINTER(RmStats)], c.c_int),
        "rm_render_sharded_runs_all": ([c.POINTER(vp), c.c_int, c.c_int, c.c_int, vp, vp, c.POINTER(RmStats)],
                                       c.c_int),
        "rm_last_error": ([vp], cp),
        "rm_status_string": ([c.c_int], cp),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    v = L.rm_abi_version()
    if v != ABI_VERSION:  # a stale build: its structs differ from the ones bound here
        raise ImportError(f"{LIB_PATH} has ABI version {v}, this binding expects {ABI_VERSION}; rebuild it")
    _LIB = L
    return L


def check(status: int, ctx=None) -> None:
    if status != RM_OK:
        msg = lib().rm_last_error(ctx).decode() if ctx else ""
        raise RmError(status, msg)
