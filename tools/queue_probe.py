#!/usr/bin/env python3
"""Do two HIP streams run kernels concurrently?  A spin kernel
(torch.cuda._sleep) on each of two streams: overlapped, the pair takes one
spin; on one hardware queue, two.  HIP maps streams onto at most
GPU_MAX_HW_QUEUES hardware queues per process (4 on the pool), sharing the
least-used queue beyond that, so two streams may serialize.  Prints one JSON
line per pair: the ratio pair_time / one_spin (1 = concurrent, 2 = serialized)."""
import ctypes
import json
import time

import torch


def spin_ms(streams, cycles):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in streams:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def cumask_stream():
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    st = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask) == 0
    return torch.cuda.ExternalStream(st.value)


def raw_stream(prio=None):
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    if prio is None:
        assert hip.hipStreamCreateWithFlags(ctypes.byref(st), ctypes.c_uint(1)) == 0
    else:
        assert hip.hipStreamCreateWithPriority(ctypes.byref(st), ctypes.c_uint(1), ctypes.c_int(prio)) == 0
    return torch.cuda.ExternalStream(st.value)


def main():
    cyc = 20_000_000
    null = torch.cuda.current_stream()
    spin_ms([null], cyc)
    one = min(spin_ms([null], cyc) for _ in range(3))
    rows = []
    pool = [torch.cuda.Stream() for _ in range(8)]
    for i, s in enumerate(pool):
        rows.append(("null+pool", i, spin_ms([null, s], cyc) / one))
    for i in range(1, 8):
        rows.append(("pool0+pool", i, spin_ms([pool[0], pool[i]], cyc) / one))
    raws = [raw_stream() for _ in range(6)]
    for i, s in enumerate(raws):
        rows.append(("null+raw", i, spin_ms([null, s], cyc) / one))
    hi = [raw_stream(-1) for _ in range(2)]
    rows.append(("null+highprio", 0, spin_ms([null, hi[0]], cyc) / one))
    rows.append(("highprio pair", 0, spin_ms(hi, cyc) / one))
    cm = [cumask_stream() for _ in range(4)]
    rows.append(("cumask pair", 0, spin_ms(cm[:2], cyc) / one))
    rows.append(("null+cumask", 0, spin_ms([null, cm[2]], cyc) / one))
    rows.append(("cumask 4", 0, spin_ms(cm, cyc) / one))
    for kind, i, ratio in rows:
        print(json.dumps({"pair": kind, "i": i, "ratio": round(ratio, 3)}), flush=True)
    print(json.dumps({"one_spin_ms": one}))


if __name__ == "__main__":
    main()
