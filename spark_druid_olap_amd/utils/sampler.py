"""Wall-clock sampling profiler over every Python thread of the process.

cProfile only sees the thread that enabled it, and a multi-threaded server (one thread per Thrift
connection) is exactly where host time matters.  ``Sampler`` wakes every ``interval`` seconds,
snapshots ``sys._current_frames()`` and counts (a) the innermost frame and (b) every frame on the
stack ("inclusive"), skipping threads that are blocked in a known wait (socket recv, lock
acquire), so the report shows where the GIL-holding time goes.

    with Sampler() as s:
        ...
    print(s.report(30))
"""
from __future__ import annotations

import collections
import sys
import threading
import time
from typing import Optional

_IDLE = ("wait", "recv", "recv_into", "accept", "select", "poll", "sleep", "get", "_wait_for_tstate_lock",
         "acquire", "readinto", "read")
# innermost Python frames that are idle inside a native call: a gateway executor blocked in
# next_batch (server/gateway.py) and a thread-pool worker blocked on its SimpleQueue
_IDLE_NATIVE = (("gateway.py", "_executor"), ("thread.py", "_worker"))


class Sampler:
    def __init__(self, interval: float = 0.0005):
        self.interval = interval
        self.self_counts = collections.Counter()
        self.incl_counts = collections.Counter()
        self.line_counts = collections.Counter()  # innermost frame at its current line
        self.samples = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @staticmethod
    def _key(f) -> str:
        c = f.f_code
        return f"{c.co_filename.rsplit('/', 2)[-1]}:{c.co_firstlineno}:{c.co_name}"

    def _run(self):
        me = threading.get_ident()
        while not self._stop.is_set():
            frames = sys._current_frames()
            for tid, f in frames.items():
                if tid == me or tid == self._starter or f is None:
                    continue
                if f.f_code.co_name in _IDLE and f.f_back is not None and \
                        f.f_code.co_filename.endswith(("threading.py", "socket.py", "queue.py", "selectors.py",
                                                       "socketserver.py")):
                    continue
                if any(f.f_code.co_name == n and f.f_code.co_filename.endswith(fn) for fn, n in _IDLE_NATIVE):
                    continue
                self.samples += 1
                self.self_counts[self._key(f)] += 1
                self.line_counts[f"{self._key(f)}@{f.f_lineno}"] += 1
                seen = set()
                while f is not None:
                    k = self._key(f)
                    if k not in seen:
                        self.incl_counts[k] += 1
                        seen.add(k)
                    f = f.f_back
            time.sleep(self.interval)

    def start(self) -> "Sampler":
        self._starter = threading.get_ident()  # the caller sleeps while sampling: not server work
        self._thread = threading.Thread(target=self._run, daemon=True, name="sdo-sampler")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def report(self, top: int = 30) -> str:
        n = max(1, self.samples)
        out = [f"{self.samples} busy-thread samples", "--- self (innermost frame)"]
        out += [f"{c / n * 100:6.1f}%  {k}" for k, c in self.self_counts.most_common(top)]
        out.append("--- self, by line")
        out += [f"{c / n * 100:6.1f}%  {k}" for k, c in self.line_counts.most_common(top)]
        out.append("--- inclusive")
        out += [f"{c / n * 100:6.1f}%  {k}" for k, c in self.incl_counts.most_common(top)]
        return "\n".join(out)
