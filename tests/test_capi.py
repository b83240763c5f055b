"""The C-ABI library (no GPU compute): it loads, exports every symbol
include/rm.h declares, and its host-side logic behaves."""
import os
import re
import subprocess

import pytest

import raymarching_amd as rm
from raymarching_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "rm.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rm_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_binding():
    assert header_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", rm.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\sT\s(rm_\w+)$", out.stdout, re.M))
    missing = set(header_symbols()) - exported
    assert not missing, missing
    L = rm.lib()
    for s in header_symbols():
        assert getattr(L, s) is not None


def test_library_has_gfx950_code_object():
    data = open(rm.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_status_strings():
    L = rm.lib()
    assert L.rm_status_string(0) == b"RM_OK"
    assert L.rm_status_string(2) == b"RM_ERR_FILE"


@pytest.mark.parametrize("H,band,n", [(4096, 16, 8), (1080, 16, 8), (1080, 27, 8), (100, 7, 3), (5, 16, 4),
                                      (8192, 16, 1), (17, 1, 17)])
def test_shard_rows_partition_the_frame(H, band, n):
    counts = [rm.shard_rows(H, band, n, s) for s in range(n)]
    assert sum(counts) == H
    # the bands are dealt round robin, so every shard owns the rows
    # {y : (y // band) % n == s}
    for s in range(n):
        assert counts[s] == sum(1 for y in range(H) if (y // band) % n == s)


def test_shard_rows_rejects_bad_arguments():
    with pytest.raises(rm.RmError):
        rm.shard_rows(0, 16, 8, 0)
    with pytest.raises(rm.RmError):
        rm.shard_rows(16, 16, 8, 8)


def test_no_gpu_means_no_context():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rm.RmError) as e:
        rm.Renderer(0)
    assert e.value.status == 5  # RM_ERR_DEVICE: no silent CPU fallback


def test_abi_version_matches_header_and_binding():
    """include/rm.h RM_ABI_VERSION, librm.so's rm_abi_version() and the ctypes
    structs of _lib.py describe the same layout (a stale build is refused)."""
    import ctypes
    txt = open(os.path.join(ROOT, "include", "rm.h")).read()
    v = int(re.search(r"#define RM_ABI_VERSION (\d+)", txt).group(1))
    assert v == _lib.ABI_VERSION == rm.lib().rm_abi_version()
    # rm_stats: 5 x 8-byte counters/ids + kernel_ms, dispatch, lat_tiles, gather_ms, deinterleave_ms
    assert ctypes.sizeof(_lib.RmStats) == 56
    assert [f[0] for f in _lib.RmStats._fields_][-4:] == ["dispatch", "lat_tiles", "gather_ms", "deinterleave_ms"]


def test_c_struct_layout_matches_binding(tmp_path):
    """The C compiler's rm_stats / rm_params layout is the one _lib.py binds."""
    import ctypes
    src = tmp_path / "layout.c"
    src.write_text('#include "rm.h"\n#include <stddef.h>\n'
                   f'_Static_assert(sizeof(rm_stats) == {ctypes.sizeof(_lib.RmStats)}, "rm_stats");\n'
                   f'_Static_assert(offsetof(rm_stats, dispatch) == {_lib.RmStats.dispatch.offset}, "dispatch");\n'
                   f'_Static_assert(offsetof(rm_stats, deinterleave_ms) == {_lib.RmStats.deinterleave_ms.offset}, "d");\n'
                   f'_Static_assert(sizeof(rm_params) == {ctypes.sizeof(_lib.RmParams)}, "rm_params");\n')
    subprocess.run(["gcc", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)], check=True)
