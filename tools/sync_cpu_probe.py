#!/usr/bin/env python3
"""Host CPU burned while a thread waits for the GPU (verdict r5 #2: the serving path's
exec_thread_cpu_ms): thread CPU time vs wall time of each wait primitive the engine uses, around
a ~20 ms device-side sleep.  ``--blocking``: the device set to blocking synchronisation
(hipSetDeviceFlags(hipDeviceScheduleBlockingSync), before any other HIP call) first.

  python tools/sync_cpu_probe.py [--blocking] [--yield]"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocking", action="store_true")
    ap.add_argument("--yield", dest="yld", action="store_true")
    ap.add_argument("--ms", type=float, default=20.0)
    a = ap.parse_args()
    if a.blocking or a.yld:
        hip = ctypes.CDLL("libamdhip64.so")
        flag = 0x4 if a.blocking else 0x2  # hipDeviceScheduleBlockingSync / hipDeviceScheduleYield
        print("hipSetDeviceFlags ->", hip.hipSetDeviceFlags(ctypes.c_uint(flag)), flush=True)
    import torch

    from spark_druid_olap_amd.ops import native

    dev = torch.device("cuda", 0)
    x = torch.ones(1, device=dev)
    torch.cuda.synchronize()
    # calibrate the device sleep
    t0 = time.perf_counter()
    torch.cuda._sleep(int(1e6))
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 1e6
    cycles = int(a.ms / 1e3 / per)

    def waits():
        yield "torch.cuda.synchronize", lambda: torch.cuda.synchronize()
        yield "stream.synchronize", lambda: torch.cuda.current_stream().synchronize()
        yield "tensor.item", lambda: x.sum().item()
        yield "native.stream_sync", lambda: native.stream_sync(dev)
        ev = torch.cuda.Event()

        def evs():
            ev.record()
            ev.synchronize()
        yield "event.synchronize", evs

    for name, w in waits():
        res = []
        for _ in range(5):
            torch.cuda._sleep(cycles)
            c0, t0 = time.thread_time(), time.perf_counter()
            w()
            res.append(((time.thread_time() - c0) * 1e3, (time.perf_counter() - t0) * 1e3))
        res.sort(key=lambda r: r[1])
        cpu, wall = res[len(res) // 2]
        print(f"{name:24s} wall {wall:7.2f} ms  thread cpu {cpu:7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
