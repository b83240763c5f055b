"""librm.so's N > 1 multi-GPU path through the C ABI, without torch in the
process (tests/rccl_standin/shard_driver): rm_comm_init_all +
rm_render_sharded_all with N contexts in one process, and rm_comm_get_id +
rm_comm_init_rank + rm_render_sharded with N processes.  Rank 0's gathered
RGBA8 frame must equal rm_render_rgba8's, byte for byte, at two poses.

On a one-GPU box real RCCL refuses two ranks on one device, so these runs put
a TEST-ONLY RCCL stand-in (tests/rccl_standin/rccl_standin.cpp, soname
librccl.so.1) on the driver's LD_LIBRARY_PATH: librm.so dlopens it exactly as
it dlopens RCCL, and every gather / send / recv librm.so issues is carried out
by it (device copies between contexts, or shared memory between processes).
Two builds cover both forms librm.so emits: ncclGather, and the grouped
ncclSend/ncclRecv form used where an RCCL lacks ncclGather.  The product never
loads the stand-in.  With two or more GPUs the same driver runs over the real
RCCL (skipped below two)."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SI = os.path.join(HERE, "rccl_standin")
DRIVER = os.path.join(SI, "build", "shard_driver")
API = ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommInitAll", "ncclCommDestroy", "ncclGroupStart",
       "ncclGroupEnd", "ncclSend", "ncclRecv", "ncclGetErrorString")


def _built():
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", SI], check=True, capture_output=True)


def run_driver(mode, n, W, H, band, scene, standin=None, one_device=True):
    _built()
    env = dict(os.environ)
    if standin:
        env["LD_LIBRARY_PATH"] = os.path.join(SI, "build", standin) + os.pathsep + env.get("LD_LIBRARY_PATH", "")
        env["RCCL_STANDIN_TIMEOUT"] = "60"
    if one_device:
        env["RM_DRIVER_ONE_DEVICE"] = "1"
    out = subprocess.run([DRIVER, mode, str(n), str(W), str(H), str(band), scene], env=env, capture_output=True,
                         text=True, timeout=150)
    assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_standin_exports_the_rccl_subset_librm_binds():
    """Both stand-in builds export what rm_comm.cpp resolves; only the gather
    build has ncclGather (the other makes librm.so take the send/recv form)."""
    _built()
    for variant, gather in (("gather", True), ("p2p", False)):
        so = os.path.join(SI, "build", variant, "librccl.so.1")
        syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
        names = {ln.split()[-1] for ln in syms.splitlines() if ln.strip()}
        assert set(API) <= names, set(API) - names
        assert ("ncclGather" in names) == gather
        assert "rccl_standin_stats" in names


def test_product_library_does_not_name_the_standin():
    lib = os.path.join(os.path.dirname(HERE), "raymarching_amd", "librm.so")
    data = open(lib, "rb").read()
    assert b"rccl_standin" not in data and b"rccl_standin" not in open(os.path.join(
        os.path.dirname(HERE), "raymarching_amd", "csrc", "rm_comm.cpp"), "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["gather", "p2p"])
@pytest.mark.parametrize("n,W,H,band,scene", [(2, 200, 120, 16, "template.frag"), (3, 131, 77, 7, "output_shader.frag"),
                                              (8, 160, 120, 8, "template.frag")])
def test_render_sharded_all_n_contexts(torch_cuda, variant, n, W, H, band, scene):
    """rm_comm_init_all + rm_render_sharded_all with n contexts (device 0): the
    group of n gathers (or n - 1 send/recv pairs) runs through the stand-in."""
    res = run_driver("all", n, W, H, band, scene, standin=variant)
    assert res["equal"] and res["frames"] == 2 and res["uses_rccl"] == 1, res
    # rm_stats of a sharded frame: render, pack + gather, and on rank 0 the de-interleave
    k, g, d = res["root_ms"]
    assert k > 0 and g > 0 and d > 0, res
    assert res["last_rank_ms"][0] > 0 and res["last_rank_ms"][2] == 0, res
    g, s, r, groups = res["standin_stats"]
    if variant == "gather":
        assert g == 2 and s == r == 0, res
    else:
        assert g == 0 and s == r == 2 * (n - 1), res
    assert groups >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["gather", "p2p"])
@pytest.mark.parametrize("n,W,H,band,scene", [(2, 200, 120, 16, "template.frag"), (3, 131, 77, 7, "output_shader.frag"),
                                              (8, 160, 120, 8, "template.frag")])
def test_render_sharded_n_processes(torch_cuda, variant, n, W, H, band, scene):
    """rm_comm_get_id + rm_comm_init_rank + rm_render_sharded, one process per
    rank (all on device 0), bands exchanged through the stand-in's shared
    memory."""
    res = run_driver("ranks", n, W, H, band, scene, standin=variant)
    assert res["equal"] and res["frames"] == 2 and res["failed_ranks"] == 0 and res["uses_rccl"] == 1, res
    k, g, d = res["root_ms"]
    assert k > 0 and g > 0 and d > 0, res
    g, s, r, _ = res["standin_stats"]  # rank 0's process
    assert (g, r) == ((2, 0) if variant == "gather" else (0, 2 * (n - 1))), res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["all", "ranks"])
@pytest.mark.parametrize("n,W,H,runs,scene", [(2, 200, 120, "25,16", "template.frag"),
                                              (3, 131, 77, "2,9,4", "output_shader.frag"),
                                              (8, 160, 120, "15,8,8,8,8,8,8,8", "template.frag")])
def test_render_sharded_runs(torch_cuda, mode, n, W, H, runs, scene):
    """rm_render_sharded_runs[_all]: weighted parts (rank r owns a run of
    runs[r] rows per cycle) gathered unpadded with grouped send/recv, the
    frame rebuilt by rm_deinterleave_cycle_rgb8, equal to rm_render_rgba8."""
    res = run_driver(mode, n, W, H, runs, scene, standin="gather")
    assert res["equal"] and res["frames"] == 2 and res["uses_rccl"] == 1, res
    k, g, d = res["root_ms"]
    assert k > 0 and g > 0 and d > 0, res
    g, s, r, _ = res["standin_stats"]
    # no ncclGather for unequal parts: every non-root part is one send/recv pair
    assert g == 0 and r == 2 * (n - 1), res


def _ngpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["all", "ranks"])
def test_real_rccl_multi_gpu(torch_cuda, mode):
    """The same driver over the real RCCL, one rank per GPU (2..8 GPUs)."""
    n = min(_ngpus(), 8)
    if n < 2:
        pytest.skip("needs two or more GPUs (RCCL refuses two ranks on one device)")
    res = run_driver(mode, n, 512, 384, 16, "template.frag", standin=None, one_device=False)
    assert res["equal"] and res["frames"] == 2 and res["uses_rccl"] == 1 and res["standin_stats"] is None, res
