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
