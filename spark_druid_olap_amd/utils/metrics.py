"""Serving metrics: per-endpoint latency percentiles, QPS and error counts ("p50/p99
latency and QPS counters in the server").

The reference leaves request metrics to Spark's UI and listener bus (``HiveThriftServer2.scala:
144-147``); a GPU server answering thousands of queries per second needs its own: every endpoint
(HiveServer2 Python server, native gateway, Druid HTTP API) records each statement's wall time
here.  Percentiles come from a fixed ring of the most recent latencies per endpoint (bounded
memory, exact over the window); QPS is measured over the last minute and since start.  Served as
JSON at ``/sparklinedata/metrics`` and in Prometheus text format at ``/metrics``.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, Optional

import numpy as np


_events: Dict[str, int] = {}
_events_lock = threading.Lock()


_event_log: list = []
_event_log_on = [False]


def count_event(name: str, n: int = 1, detail: Optional[str] = None) -> None:
    """Process-wide event counter (device-memory releases, statement retries, P2P fallbacks, plan
    and kernel swaps).  With ``log_events(True)`` every event is also kept with its time
    (``time.perf_counter``): the serving timeline lines them up with stalls."""
    with _events_lock:
        _events[name] = _events.get(name, 0) + n
        if _event_log_on[0] and len(_event_log) < 100_000:
            _event_log.append((time.perf_counter(), name) if detail is None else
                              (time.perf_counter(), name, detail[:160]))


def log_events(on: bool) -> list:
    """Start (clearing) or stop the timed event log; returns the events logged so far."""
    with _events_lock:
        out = list(_event_log)
        if on:
            _event_log.clear()
        _event_log_on[0] = on
        return out


def events() -> Dict[str, int]:
    with _events_lock:
        return dict(_events)


class _Series:
    __slots__ = ("lat", "ts", "n", "errors", "total_ms")

    def __init__(self, window: int):
        self.lat = np.zeros(window, dtype=np.float64)   # ms, ring buffer
        self.ts = np.zeros(window, dtype=np.float64)    # completion times (monotonic s)
        self.n = 0
        self.errors = 0
        self.total_ms = 0.0


class ServerMetrics:
    def __init__(self, window: int = 8192):
        self.window = int(window)
        self._lock = threading.Lock()
        self._series: Dict[str, _Series] = {}
        self.started = time.monotonic()

    def record(self, endpoint: str, ms: float, ok: bool = True, count: int = 1) -> None:
        """``count`` identical statements answered by one execution (batched) share its latency."""
        now = time.monotonic()
        with self._lock:
            s = self._series.get(endpoint)
            if s is None:
                s = self._series[endpoint] = _Series(self.window)
            for _ in range(max(1, int(count))):
                i = s.n % self.window
                s.lat[i] = ms
                s.ts[i] = now
                s.n += 1
                s.total_ms += ms
                if not ok:
                    s.errors += 1

    def time(self, endpoint: str):
        """``with metrics.time("thrift"):`` records the block's wall time (an exception = error)."""
        return _Timer(self, endpoint)

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        now = time.monotonic()
        out = {}
        with self._lock:
            for ep, s in self._series.items():
                k = min(s.n, self.window)
                lat = s.lat[:k] if s.n <= self.window else s.lat
                ts = s.ts[:k] if s.n <= self.window else s.ts
                p50, p95, p99 = (np.percentile(lat, [50, 95, 99]).tolist() if k else [0.0, 0.0, 0.0])
                recent = int((ts >= now - 60.0).sum()) if k else 0
                span = min(60.0, max(1e-9, now - self.started))
                out[ep] = {"count": s.n, "errors": s.errors, "p50_ms": p50, "p95_ms": p95, "p99_ms": p99,
                           "max_ms": float(lat.max()) if k else 0.0, "mean_ms": s.total_ms / max(1, s.n),
                           "qps_1m": recent / span, "qps_total": s.n / max(1e-9, now - self.started)}
        return out

    def prometheus(self) -> str:
        lines = []
        for name, help_, key in (("sdo_requests_total", "statements answered", "count"),
                                 ("sdo_request_errors_total", "statements that failed", "errors"),
                                 ("sdo_qps_1m", "statements per second over the last minute", "qps_1m")):
            lines += [f"# HELP {name} {help_}", f"# TYPE {name} {'counter' if 'total' in name else 'gauge'}"]
            for ep, v in sorted(self.snapshot().items()):
                lines.append(f'{name}{{endpoint="{ep}"}} {v[key]}')
        lines += ["# HELP sdo_latency_ms statement latency percentiles over the recent window",
                  "# TYPE sdo_latency_ms summary"]
        for ep, v in sorted(self.snapshot().items()):
            for q, key in (("0.5", "p50_ms"), ("0.95", "p95_ms"), ("0.99", "p99_ms")):
                lines.append(f'sdo_latency_ms{{endpoint="{ep}",quantile="{q}"}} {v[key]}')
            lines.append(f'sdo_latency_ms_count{{endpoint="{ep}"}} {v["count"]}')
        lines += ["# HELP sdo_events_total process events (memory releases, retries)", "# TYPE sdo_events_total counter"]
        for k, v in sorted(events().items()):
            lines.append(f'sdo_events_total{{event="{k}"}} {v}')
        return "\n".join(lines) + "\n"


class _Timer:
    def __init__(self, m: ServerMetrics, ep: str):
        self.m, self.ep = m, ep

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, et, ev, tb):
        self.m.record(self.ep, (time.perf_counter() - self.t0) * 1e3, ok=et is None)
        return False


_GLOBAL: Optional[ServerMetrics] = None


def metrics_of(session) -> ServerMetrics:
    """The metrics registry shared by a session and its client-session views."""
    m = getattr(session, "metrics", None)
    if m is None:
        global _GLOBAL
        if _GLOBAL is None:
            _GLOBAL = ServerMetrics()
        m = _GLOBAL
    return m
