"""Publishing device artifacts to caches shared across execution slots.

Every execution slot (engine/scheduler.py, server/spmd.py) runs its statements on its own HIP
stream, and PyTorch's streams do not synchronise with each other.  Lowering and finalize build
device-side artifacts lazily and cache them for every later statement: bit-packed column copies
(segment/packed.py), u16 HLL code planes (segment/hllcode.py), functional-dependency tables and
per-dictionary LUTs (engine/lower.py), decode tables (engine/partials.py).  The thread that builds
one enqueues the kernels on ITS current stream; a statement on another slot that finds the cache
entry launches its scan on ITS stream right away -- and can read the table before the producing
kernels ran (garbage ids feeding group keys and table indices: an out-of-bounds access).  A lease
orders the slot's stream after the default stream when it starts, which does not cover artifacts
published later by another thread (a statement re-prepared while others run: engine/device_exec.py
async_compile).  So a builder completes its work before the artifact becomes visible."""
from __future__ import annotations

import torch


def publish(x, dev):
    """``x`` (the value about to enter a shared cache), after the current stream of ``dev`` --
    which produced it -- has drained.  A one-time cost per artifact; a no-op off the GPU."""
    if x is not None and dev is not None and torch.device(dev).type == "cuda":
        torch.cuda.current_stream(torch.device(dev)).synchronize()
    return x
