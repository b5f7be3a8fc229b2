"""How a thread waits for the GPU.

The HIP runtime's default wait spins: a thread blocked in a stream / event synchronisation or a
device-to-host copy burns its core for the whole wait (tools/sync_cpu_probe.py on MI355X: 5.1 ms
of thread CPU per 5.1 ms wait, every primitive the engine uses).  A single-query benchmark wants
exactly that (the lowest wake-up latency), a server does not: its executor threads wait on
partitioned group-bys for tens of milliseconds each, and the spinning cores are the ones its Thrift
clients, compile threads and gateway need (``exec_thread_cpu_ms`` of tools/concurrency_bench.py).
``hipDeviceScheduleBlockingSync`` makes those waits sleep on the completion interrupt instead
(0.3 ms of CPU per wait, profiles/r6/sync_cpu_probe.txt) -- but every wake-up then comes late: at
400 QPS of the BI plan the server's capacity fell below the offered load (382/s, p99 2.3 s vs
126 ms spinning).  The engine's own waits therefore spin for 2 ms and then sleep between polls
(ops/csrc/bindings.cpp wait_stream), and the servers keep HIP's spin mode by default.  The flag is
per device and only takes before the process's first HIP call touches the device, so server entry
points set it first thing when asked to.
"""
from __future__ import annotations

import ctypes
from typing import Optional

HIP_DEVICE_SCHEDULE_SPIN = 0x1
HIP_DEVICE_SCHEDULE_YIELD = 0x2
HIP_DEVICE_SCHEDULE_BLOCKING_SYNC = 0x4

_MODES = {"spin": HIP_DEVICE_SCHEDULE_SPIN, "yield": HIP_DEVICE_SCHEDULE_YIELD,
          "blocking": HIP_DEVICE_SCHEDULE_BLOCKING_SYNC}
_applied: dict = {}


def set_wait_mode(mode: str = "blocking", device: Optional[int] = None) -> bool:
    """Set how this process's threads wait for ``device`` (default: the current one): "blocking"
    (sleep on the interrupt), "spin" or "yield".  Call before anything else uses the GPU (torch
    included); returns False when there is no HIP runtime or it refused (already initialised)."""
    if mode not in _MODES:
        raise ValueError(f"wait mode {mode!r}: one of {sorted(_MODES)}")
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return False
    if device is not None and hip.hipSetDevice(ctypes.c_int(int(device))) != 0:
        return False
    ok = hip.hipSetDeviceFlags(ctypes.c_uint(_MODES[mode])) == 0
    if ok:
        _applied[device] = mode
    return ok


def wait_mode() -> dict:
    """The modes this process set, per device (None: the current device at the time)."""
    return dict(_applied)
