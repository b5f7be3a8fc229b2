"""Host memory tuning for the result path.

Query results are a handful of multi-MB numpy arrays per query (e.g. a 1.2M-group TPC-H Q3).
With glibc defaults every such array is its own ``mmap`` and freeing it ``munmap``s and later
re-faults pages -- a few milliseconds of page-table work billed to whichever query happens to drop
the previous result.  Raising the mmap threshold to glibc's maximum (32 MB) and disabling heap
trimming keeps those buffers in the process heap for reuse."""
from __future__ import annotations

import ctypes
import ctypes.util
import os

_DONE = False
M_TRIM_THRESHOLD = -1
M_MMAP_THRESHOLD = -3


def tune_host_malloc() -> bool:
    global _DONE
    if _DONE:
        return False
    _DONE = True
    try:
        libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6")
        ok1 = libc.mallopt(M_MMAP_THRESHOLD, 32 << 20)
        ok2 = libc.mallopt(M_TRIM_THRESHOLD, 1 << 30)
        return bool(ok1 and ok2)
    except (OSError, AttributeError):
        return False


def serving_gc() -> None:
    """Garbage-collector settings for a long-running server process: everything allocated so far
    (datasources, dictionaries, plan caches, imported modules) moves to the permanent generation
    (``gc.freeze``) and the young-generation threshold is raised, so a full collection no longer
    walks millions of long-lived objects in the middle of a statement (a multi-hundred-millisecond
    pause at the p99 of a many-client run)."""
    import gc

    gc.collect()
    gc.freeze()
    gc.set_threshold(50_000, 50, 100)


SERVING_ALLOC_CONF = "garbage_collection_threshold:0.7"


def serving_allocator_conf() -> bool:
    """A serving process's caching-allocator settings (call before the process's first device
    allocation; a user's own ``PYTORCH_HIP_ALLOC_CONF`` / ``PYTORCH_CUDA_ALLOC_CONF`` wins).

    Above 70 % of the device the allocator returns its least recently used free blocks a few at a
    time instead of letting reserved memory reach the cap, where it frees EVERY cached block with
    the device synchronised and retries -- the cold BI burst's 3.3 s freeze of every slot
    (profiles/r6/cold_burst_notes.md).  Same-box A/B, cold closed loop, 64 clients, 8 slots:
    575-579 exec/s and p99 187-188 ms with no retry, against 461-488 exec/s and p99 256-261 ms with
    one (profiles/r6/thrift_jmx_cold_alloc_gc_ab.txt)."""
    if os.environ.get("PYTORCH_HIP_ALLOC_CONF") or os.environ.get("PYTORCH_CUDA_ALLOC_CONF"):
        return False
    os.environ["PYTORCH_HIP_ALLOC_CONF"] = SERVING_ALLOC_CONF
    return True


RUNTIME_RESERVE = int(os.environ.get("SDO_RUNTIME_RESERVE_GB", "8")) << 30


def reserve_runtime_memory(device=None) -> float:
    """Cap the torch caching allocator below the device size, leaving ``RUNTIME_RESERVE`` bytes to
    the HIP runtime's own allocations (kernel scratch, loaded code objects, RCCL buffers).  Those
    are made outside torch: a serving process whose cache has grown over the whole device gets a
    scratch allocation failure, which aborts the HIP queue -- every later statement fails.  With
    the cap torch raises an out-of-memory error first, which the engine answers by evicting cached
    scan buffers (engine/device_exec.py _with_eviction) or fails that one statement.  Returns the
    fraction set (0 when there is no GPU)."""
    import torch

    if not torch.cuda.is_available() or RUNTIME_RESERVE <= 0:
        return 0.0
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    total = torch.cuda.get_device_properties(dev).total_memory
    frac = max(0.5, 1.0 - RUNTIME_RESERVE / total)
    torch.cuda.set_per_process_memory_fraction(frac, dev)
    return frac
