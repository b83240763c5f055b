#!/usr/bin/env python3
"""SIMD-efficiency model of lane-per-pixel vs wave-compacted schedules.

Uses the oracle's per-pixel sequence of sceneSDF segments (march, normal,
AO, shadow, SSS) to estimate, per 64-lane wave:
  direct:   sum over code positions of the max lane count (structured loops)
  compact:  lanes pull pixels from a per-wave queue of K pixels and every
            iteration evaluates one step on every busy lane
efficiency = useful lane-steps / (64 x wave iterations).
"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import oracle  # noqa: E402
from raymarching_amd import POSES  # noqa: E402

TEMPLATES = {"T": [0, 1, 0, 2, 3], "O": [0, 1, 2, 3, 4, 0, 1, 2, 3, 4], "S0": [0, 1]}


def segments(scene, W, H, pose, steps):
    L = oracle.lib()
    u = oracle.uniforms(W, H, pos=pose["pos"], mouse=pose["mouse"], time=pose["time"], max_steps=steps)
    seg = np.zeros((H, W, 24, 2), np.uint16)
    ns = np.zeros((H, W), np.uint8)
    L.oracle_render_segments.argtypes = [ctypes.c_int, ctypes.POINTER(oracle.OracleUniforms), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_render_segments(oracle.SCENES[scene], ctypes.byref(u), W, H, 0, H, seg.ctypes.data, ns.ctypes.data)
    return seg, ns


def aligned(seg, ns, tmpl):
    """[H, W, len(tmpl)] counts aligned to the scene's code positions."""
    H, W = ns.shape
    out = np.zeros((H, W, len(tmpl)), np.int64)
    for y in range(H):
        for x in range(W):
            k = 0
            for i in range(ns[y, x]):
                ph, c = seg[y, x, i]
                while k < len(tmpl) and tmpl[k] != ph:
                    k += 1
                if k < len(tmpl):
                    out[y, x, k] += c
                    k += 1
    return out


def tiles(a, t=8):
    H, W = a.shape[:2]
    a = a[: H // t * t, : W // t * t]
    return a.reshape(H // t, t, W // t, t, *a.shape[2:]).swapaxes(1, 2).reshape(-1, t * t, *a.shape[2:])


def direct_eff(al):
    w = tiles(al)  # [nwaves, 64, npos]
    useful = w.sum()
    cost = w.max(axis=1).sum() * 64
    return useful / cost


def compact_eff(tot, K):
    w = tiles(tot).reshape(-1)  # pixel costs in tile order
    n = len(w) // K * K
    useful, cost = 0, 0
    for b in range(0, n, K):
        q = w[b:b + K]
        lanes = np.zeros(64)
        for c in q:  # greedy: next pixel to the lane that frees first
            i = lanes.argmin()
            lanes[i] += c
        useful += q.sum()
        cost += lanes.max() * 64
    return useful / cost


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "T"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    for pn in (sys.argv[4].split(",") if len(sys.argv) > 4 else ["P0"]):
        seg, ns = segments(scene, W, W, POSES[pn], steps)
        al = aligned(seg, ns, TEMPLATES[scene])
        tot = al.sum(-1)
        res = {"pose": pn, "evals/px": float(tot.mean()), "direct": direct_eff(al)}
        for K in (64, 256, 1024, 4096):
            res[f"compact{K}"] = compact_eff(tot, K)
        print(scene, W, {k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()


def band_main(scene, W, steps, pn, row0, nrows):
    """Same model on a band of rows of a full-size frame."""
    L = oracle.lib()
    pose = POSES[pn]
    u = oracle.uniforms(W, W, pos=pose["pos"], mouse=pose["mouse"], time=pose["time"], max_steps=steps)
    seg = np.zeros((nrows, W, 24, 2), np.uint16)
    ns = np.zeros((nrows, W), np.uint8)
    L.oracle_render_segments.argtypes = [ctypes.c_int, ctypes.POINTER(oracle.OracleUniforms), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_render_segments(oracle.SCENES[scene], ctypes.byref(u), W, W, row0, nrows, seg.ctypes.data,
                             ns.ctypes.data)
    al = aligned(seg, ns, TEMPLATES[scene])
    tot = al.sum(-1)
    res = {"pose": pn, "rows": f"{row0}+{nrows}", "evals/px": float(tot.mean()), "direct": direct_eff(al)}
    for K in (64, 256, 1024):
        res[f"compact{K}"] = compact_eff(tot, K)
    print(scene, W, {k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}, flush=True)


# ---------------------------------------------------------------- per phase
PHASE_NAMES = {"O": ["march", "normal", "AO", "shadow", "SSS", "refl.march", "refl.normal", "refl.AO",
                     "refl.shadow", "refl.SSS"],
               "T": ["march", "normal", "refl.march", "AO", "shadow"], "S0": ["march", "normal"]}


def aligned_np(seg, ns, tmpl):
    """aligned() vectorized: [..., len(tmpl)] counts per code position."""
    P = len(tmpl)
    nxt = np.full((P + 1, 8), P, np.int64)  # next position >= k holding phase ph
    for k in range(P - 1, -1, -1):
        nxt[k] = nxt[k + 1]
        nxt[k, tmpl[k]] = k
    shp = ns.shape
    seg = seg.reshape(-1, seg.shape[-2], 2)
    ns = ns.reshape(-1)
    out = np.zeros((len(ns), P + 1), np.int64)
    k = np.zeros(len(ns), np.int64)
    rows = np.arange(len(ns))
    for i in range(seg.shape[1]):
        live = i < ns
        ph = seg[:, i, 0].astype(np.int64)
        c = seg[:, i, 1].astype(np.int64)
        pos = nxt[np.minimum(k, P), ph]
        pos = np.where(live, pos, P)
        np.add.at(out, (rows, pos), np.where(live, c, 0))
        k = np.where(live & (pos < P), pos + 1, k)
    return out[:, :P].reshape(*shp, P)


def phase_report(scene, W, steps, pn, bands, rows_per_band=64):
    """Lane utilization per code position of the one-wave 8x8 tiles, over
    `bands` row bands spread over a W x W frame: useful lane-steps / (64 x the
    wave's longest lane), and the lanes that reach each phase among the waves
    that run it (the shading code of that phase runs at that utilization)."""
    L = oracle.lib()
    pose = POSES[pn]
    u = oracle.uniforms(W, W, pos=pose["pos"], mouse=pose["mouse"], time=pose["time"], max_steps=steps)
    L.oracle_render_segments.argtypes = [ctypes.c_int, ctypes.POINTER(oracle.OracleUniforms), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    tmpl = TEMPLATES[scene]
    acc = []
    for b in range(bands):
        row0 = (W // bands * b + W // (2 * bands)) // 8 * 8
        seg = np.zeros((rows_per_band, W, 24, 2), np.uint16)
        ns = np.zeros((rows_per_band, W), np.uint8)
        L.oracle_render_segments(oracle.SCENES[scene], ctypes.byref(u), W, W, row0, rows_per_band, seg.ctypes.data,
                                 ns.ctypes.data)
        acc.append(tiles(aligned_np(seg, ns, tmpl)))
    w = np.concatenate(acc)  # [nwaves, 64, P]
    useful = w.sum(axis=(0, 1))
    cost = w.max(axis=1).sum(axis=0) * 64
    reach = (w > 0)
    waves_run = reach.any(axis=1)  # [nwaves, P]
    lanes_reach = reach.sum(axis=1)
    names = PHASE_NAMES.get(scene, [str(k) for k in range(len(tmpl))])
    out = {"scene": scene, "W": W, "steps": steps, "pose": pn, "waves": int(len(w)),
           "evals/px": round(float(w.sum() / (len(w) * 64)), 2), "direct": round(float(useful.sum() / cost.sum()), 4),
           "phases": {}}
    for k, nm in enumerate(names):
        nrun = int(waves_run[:, k].sum())
        out["phases"][nm] = {
            "evals_share": round(float(useful[k] / useful.sum()), 4),
            "step_util": round(float(useful[k] / max(cost[k], 1)), 4),
            "lane_util": round(float(lanes_reach[:, k][waves_run[:, k]].sum() / max(64 * nrun, 1)), 4),
            "waves_run": round(nrun / len(w), 4)}
    return out
