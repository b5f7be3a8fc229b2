"""Query cancellation and deadlines.

The reference relays Spark task kills to in-flight Druid HTTP requests through a polling
watchdog (``TaskCancelHandler``, ``sd/DruidRDD.scala:428-493``).  In-process, a query is a short
sequence of fused GPU scans plus host operators, so a token checked between operators (and before
every GPU launch) gives prompt cancellation without aborting a kernel mid-flight.  Deadlines come
from ``spark.sparklinedata.druid.query.timeout.ms`` or the Thrift ``queryTimeout``."""
from __future__ import annotations

import threading
import time
from typing import Optional

from .errors import QueryCancelled, QueryTimeout


class CancelToken:
    def __init__(self, timeout_ms: Optional[float] = None):
        self._ev = threading.Event()
        self.deadline = time.monotonic() + timeout_ms / 1e3 if timeout_ms else None
        self.reason = ""

    def cancel(self, reason: str = "cancelled") -> None:
        self.reason = reason
        self._ev.set()

    @property
    def cancelled(self) -> bool:
        return self._ev.is_set()

    def check(self) -> None:
        if self._ev.is_set():
            raise QueryCancelled(self.reason or "query cancelled")
        if self.deadline is not None and time.monotonic() > self.deadline:
            raise QueryTimeout("query exceeded its deadline")


# ------------------------------------------------------------------------------------------------
# The calling thread's current token: executors enter ``scope(token)`` around a statement and the
# engine calls ``checkpoint()`` at its stage boundaries (before each scan / segment batch, between
# the stages of a nested query), so a cancel or deadline stops a running query within one kernel
# (ms) -- the GPU analogue of the reference's watchdog aborting in-flight Druid HTTP requests
# (sd/DruidRDD.scala:428-493).  Across ranks, the pre-scan checkpoint sits inside the merge's
# failure agreement (parallel/fault.py), so every rank aborts the query together.
_tls = threading.local()


class scope:
    def __init__(self, token: Optional[CancelToken]):
        self.token = token

    def __enter__(self):
        self.prev = getattr(_tls, "token", None)
        _tls.token = self.token if self.token is not None else self.prev
        return self.token

    def __exit__(self, *exc):
        _tls.token = self.prev
        return False


def current() -> Optional[CancelToken]:
    return getattr(_tls, "token", None)


def checkpoint() -> None:
    t = getattr(_tls, "token", None)
    if t is not None:
        t.check()
