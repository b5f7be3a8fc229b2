"""Tracing: roctx ranges around every query stage + an in-process per-query timeline.

The reference's tracing is log-based (``spark.sparklinedata.druid.debug.transformations``,
``asd/DruidTransforms.scala:121-136``; per-request timings ``sd/client/DruidClient.scala:235-277``;
SURVEY §5.1).  On MI355X the stages of a query (parse/plan, lower, scan kernel, merge collective,
finalize/D2H, host post-processing) are bracketed with roctx ranges (``roctxRangePushA`` /
``roctxRangePop`` from ``librocprofiler-sdk-roctx``) so ``rocprofv3 --marker-trace --kernel-trace``
shows them on the same timeline as the HIP kernels and RCCL collectives, and the same ranges are
recorded host-side per thread (``Timeline``) for ``EXPLAIN``-style breakdowns without a profiler.

Enabled with ``SDO_TRACE=1`` (or ``enable()``); disabled it costs one attribute check per stage.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time
from typing import List, Optional, Tuple

_LIB = None
_ENABLED = os.environ.get("SDO_TRACE", "0") not in ("0", "", "false")
_TL = threading.local()


def _lib():
    global _LIB
    if _LIB is None:
        _LIB = False
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                     "libroctx64.so"):
            for d in ("", "/opt/rocm/lib/"):
                try:
                    lib = ctypes.CDLL(d + name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _LIB = lib
                    return _LIB
                except (OSError, AttributeError):
                    continue
    return _LIB


def enable(on: bool = True) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def available() -> bool:
    return bool(_lib())


class Timeline:
    """Host-side record of (stage, start_s, end_s, depth) for the current thread's query."""

    def __init__(self):
        self.events: List[Tuple[str, float, float, int]] = []
        self.depth = 0

    def summary(self) -> List[Tuple[str, float]]:
        return [(("  " * d) + n, (b - a) * 1e3) for n, a, b, d in self.events]


def timeline() -> Timeline:
    t = getattr(_TL, "tl", None)
    if t is None:
        t = _TL.tl = Timeline()
    return t


def reset() -> Timeline:
    _TL.tl = Timeline()
    return _TL.tl


_NOOP = contextlib.nullcontext()


def span(name: str):
    """roctx range + timeline entry (no-op unless tracing is enabled).  Disabled, it returns one
    shared null context: no generator per call (a few of these wrap every query's hot path)."""
    if not _ENABLED:
        return _NOOP
    return _span(name)


@contextlib.contextmanager
def _span(name: str):
    lib = _lib()
    tl = timeline()
    if lib:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    tl.depth += 1
    try:
        yield
    finally:
        tl.depth -= 1
        tl.events.append((name, t0, time.perf_counter(), tl.depth))
        if lib:
            lib.roctxRangePop()


def mark(msg: str) -> None:
    if _ENABLED and _lib():
        _lib().roctxMarkA(msg.encode())
