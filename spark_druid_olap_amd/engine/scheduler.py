"""Concurrent query execution on one GPU: stream slots, admission control and batching of
identical statements.

The reference serves many BI clients at once through a pooled HTTP client (100 connections, 20 per
route, ``asd/DruidPlanner.scala:83-90``) in front of Druid's processing-thread pools, driven in its
BI benchmark by JMeter threads on a fair scheduler pool (``docs/bi-benchmark/snap-sales-demo.jmx:
87-101``).  On one MI355X the equivalent resources are HIP streams and the device buffers a query
writes into:

* ``StreamScheduler`` owns K *slots*.  A slot is one HIP stream plus the right to use the slot's
  device arena (accumulators, hash tables, HLL registers -- see ``engine/device_exec.py``
  ``SlotArena``, which every prepared scan run on ``current_slot()`` carves its buffers from).  A
  statement leases a slot for its whole execution, so two clients running the same prepared query
  never share accumulators, and their kernels overlap on different streams.  Leasing blocks when
  all K slots are busy: that is the admission queue.  Each lease starts a new *statement epoch* of
  the slot (``slot_epoch``): the arena's bump allocation restarts, so the slot's device memory is
  its largest statement's need, not the sum over every prepared plan ever run on it.
* ``Coalescer`` batches identical statements that are *waiting* for a slot: the first becomes the
  leader, later arrivals with the same key attach to it, and when the leader gets a slot it executes
  once for all of them (a shared scan).  A statement that arrives after the leader started executing
  opens a new batch -- nothing is served from a result computed before the request arrived.

Slot 0 is the implicit slot of unscheduled callers (scripts, benchmarks, tests); scheduled work uses
slots 1..K.
"""
from __future__ import annotations

import contextlib
import queue
import threading
import time
from typing import Any, Callable, Dict, Hashable, Optional

import torch

_ctx = threading.local()


def current_slot() -> int:
    """Buffer slot of the calling thread's current execution (0 = unscheduled)."""
    return getattr(_ctx, "slot", 0)


_epochs: Dict[int, int] = {}


def slot_epoch(slot: int) -> int:
    """Statement counter of a slot: bumped each time a statement starts on it (``use_slot``)."""
    return _epochs.get(slot, 0)


@contextlib.contextmanager
def use_slot(slot: int):
    """Run the calling thread's statement on ``slot`` (one statement per slot at a time: the
    scheduler's lease or the SPMD slot worker guarantees it)."""
    prev = getattr(_ctx, "slot", 0)
    _ctx.slot = slot
    _epochs[slot] = _epochs.get(slot, 0) + 1
    try:
        yield slot
    finally:
        _ctx.slot = prev


class StreamScheduler:
    """K execution slots, each a HIP stream; ``lease()`` blocks while all are busy."""

    def __init__(self, slots: int = 4, device: Optional[torch.device] = None):
        self.nslots = max(1, int(slots))
        self.device = device
        self._free: "queue.Queue[int]" = queue.Queue()
        for s in range(1, self.nslots + 1):
            self._free.put(s)
        self._streams: Dict[int, Any] = {}
        self._lock = threading.Lock()
        self.stats = {"leases": 0, "wait_ms": 0.0, "max_wait_ms": 0.0}

    def _stream(self, slot: int):
        if self.device is None or self.device.type != "cuda":
            return None
        with self._lock:
            s = self._streams.get(slot)
            if s is None:
                s = self._streams[slot] = torch.cuda.Stream(self.device)
            return s

    @contextlib.contextmanager
    def lease(self):
        t0 = time.perf_counter()
        slot = self._free.get()
        w = (time.perf_counter() - t0) * 1e3
        with self._lock:
            self.stats["leases"] += 1
            self.stats["wait_ms"] += w
            self.stats["max_wait_ms"] = max(self.stats["max_wait_ms"], w)
        try:
            st = self._stream(slot)
            with use_slot(slot):
                if st is None:
                    yield slot
                else:
                    # work the statement's preparation launched on the default stream (lowering:
                    # HLL code planes, FD tables) precedes the slot's kernels
                    st.wait_stream(torch.cuda.default_stream(st.device))
                    with torch.cuda.stream(st):
                        yield slot
                    _sync(st)
        finally:
            self._free.put(slot)


def _sync(st) -> None:
    """The slot stream's end-of-statement wait: the native extension's spin-then-sleep wait when it
    is loaded (ops/csrc/bindings.cpp wait_stream: a long statement does not spin a core)."""
    from ..ops import native

    m = native.loaded()
    if m is not None:
        m.stream_sync(st.cuda_stream)
    else:
        st.synchronize()


class _Flight:
    __slots__ = ("event", "result", "error", "started", "joined")

    def __init__(self):
        self.event = threading.Event()
        self.result = None
        self.error: Optional[BaseException] = None
        self.started = False
        self.joined = 0


class Coalescer:
    """Run ``fn`` once for every identical request queued together (see module docstring)."""

    def __init__(self, scheduler: StreamScheduler):
        self.scheduler = scheduler
        self._lock = threading.Lock()
        self._waiting: Dict[Hashable, _Flight] = {}
        self.stats = {"executions": 0, "coalesced": 0}

    def run(self, key: Optional[Hashable], fn: Callable[[], Any]) -> Any:
        if key is None:
            with self.scheduler.lease():
                return fn()
        with self._lock:
            f = self._waiting.get(key)
            leader = f is None
            if leader:
                f = self._waiting[key] = _Flight()
            else:
                f.joined += 1
                self.stats["coalesced"] += 1
        if not leader:
            f.event.wait()
            if f.error is not None:
                raise f.error
            return f.result
        try:
            with self.scheduler.lease():
                with self._lock:
                    # later arrivals open a new batch from here on
                    f.started = True
                    if self._waiting.get(key) is f:
                        del self._waiting[key]
                    self.stats["executions"] += 1
                f.result = fn()
        except BaseException as e:  # noqa: BLE001  (every waiter sees the leader's error)
            f.error = e
            with self._lock:
                if self._waiting.get(key) is f:
                    del self._waiting[key]
            raise
        finally:
            f.event.set()
        return f.result
