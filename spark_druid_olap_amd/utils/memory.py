"""Host memory tuning for the result path.

Query results are a handful of multi-MB numpy arrays per query (e.g. a 1.2M-group TPC-H Q3).
With glibc defaults every such array is its own ``mmap`` and freeing it ``munmap``s and later
re-faults pages -- a few milliseconds of page-table work billed to whichever query happens to drop
the previous result.  Raising the mmap threshold to glibc's maximum (32 MB) and disabling heap
trimming keeps those buffers in the process heap for reuse.  Opt out with ``SDO_NO_MALLOPT=1``."""
from __future__ import annotations

import ctypes
import ctypes.util
import os

_DONE = False
M_TRIM_THRESHOLD = -1
M_MMAP_THRESHOLD = -3


def tune_host_malloc() -> bool:
    global _DONE
    if _DONE or os.environ.get("SDO_NO_MALLOPT"):
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
