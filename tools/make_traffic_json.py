#!/usr/bin/env python3
"""profiles/pmc_counters.json entry from a tools/pmc_profile.sh summary (the
counters bench.py's roofline reads for its workload).

Per launch of the render kernel:
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (KiB counters; on
      gfx950 FETCH_SIZE reads half the bytes of wide coalesced reads,
      MI355X_MICROARCH.md "HBM"; WRITE_SIZE is exact for the RGBA8 stores,
      checked against the 64 MiB frame)
  flop_exec = 64 * (ADD + MUL + TRANS + 2 * FMA) executed F32 wave-instructions
      (issued lane slots: 64 per wave-instruction whatever the exec mask)
  active_lane_frac = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU): the
      mean fraction of a VALU instruction's lanes that are active (exec mask)
  flop_lanes = flop_exec * active_lane_frac: FP32 FLOP done by active lanes
  clock_hz = GRBM_GUI_ACTIVE / 8 XCDs / the kernel's average duration (from
      the kernel-trace stats of the same command)
  render_code_hash = rm_render_code_hash() of the library in the tree (the
      build whose launch was counted: run this where the profile ran, with
      the same librm.so)
  executed_ray_steps_per_launch = config.executed_ray_steps_per_frame of the
      bench line the same command printed (BENCH_LOG: a file whose last JSON
      line is bench.py's), so bench.py can price a rank's share of the frame
      (N > 1) or a walk's poses per executed ray-step
usage: make_traffic_json.py SUMMARY.json KEY KERNEL_SUBSTR KERNEL_STATS.csv [OUT] [BENCH_LOG]
"""
import csv
import json
import os
import sys

summ, key, ksub, stats = sys.argv[1:5]
out = sys.argv[5] if len(sys.argv) > 5 and sys.argv[5] else "profiles/pmc_counters.json"
bench_log = sys.argv[6] if len(sys.argv) > 6 else None
d = json.load(open(summ))
k = [n for n in d if ksub in n][0]
v = d[k]
avg_ns = [float(r["AverageNs"]) for r in csv.DictReader(open(stats)) if ksub in r["Name"]][0]
entry = {"kernel": k, "source": os.path.relpath(summ), "kernel_stats": os.path.relpath(stats),
         "avg_kernel_ns_trace": avg_ns}
try:  # the build these counters were taken with (bench.py prices a launch with them only on a match)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import raymarching_amd as rm
    entry["render_code_hash"] = rm.render_code_hash()
except Exception as e:  # noqa: BLE001 (the library is not built here: no hash, bench falls back to the duration check)
    print("no render code hash:", e, file=sys.stderr)
if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
    entry.update(FETCH_SIZE_KiB=v["FETCH_SIZE"], WRITE_SIZE_KiB=v["WRITE_SIZE"],
                 hbm_bytes_per_launch=(2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024)
for c in ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVES", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_INSTS_BRANCH",
          "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F32",
          "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES"):
    if c in v:
        entry[c] = v[c]
f32 = ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F32")
if all(c in v for c in f32):
    entry["flop_exec_per_launch"] = 64 * (v[f32[0]] + v[f32[1]] + v[f32[2]] + 2 * v[f32[3]])
if "SQ_THREAD_CYCLES_VALU" in v and "SQ_ACTIVE_INST_VALU" in v:
    entry["active_lane_frac"] = v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"])
    if "flop_exec_per_launch" in entry:
        entry["flop_lanes_per_launch"] = entry["flop_exec_per_launch"] * entry["active_lane_frac"]
if bench_log:
    line = [ln for ln in open(bench_log) if ln.startswith("{") and '"metric"' in ln][-1]
    entry["executed_ray_steps_per_launch"] = int(json.loads(line)["config"]["executed_ray_steps_per_frame"])
    entry["executed_ray_steps_source"] = os.path.relpath(bench_log)
if "GRBM_GUI_ACTIVE" in v:
    entry["clock_hz"] = v["GRBM_GUI_ACTIVE"] / 8 / (avg_ns * 1e-9)
allj = json.load(open(out)) if os.path.exists(out) else {}
allj[key] = entry
json.dump(allj, open(out, "w"), indent=1)
print(key, json.dumps(entry))
