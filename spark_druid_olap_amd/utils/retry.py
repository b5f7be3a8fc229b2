"""Retry helpers (``sd/RetryUtils.scala:28-108``): fixed-delay ``retry_until``, exponential backoff
``exec_with_backoff`` / ``retry_on_errors`` (start 200 ms, cap 5 s).  Used for ingestion-task
polling, index bootstrap in tests, and the HTTP client."""
from __future__ import annotations

import random
import time
from typing import Callable, Optional, Tuple, Type, TypeVar

T = TypeVar("T")


class RetryTimeout(TimeoutError):
    pass


def retry_until(fn: Callable[[], T], done: Callable[[T], bool], timeout_s: float = 60.0,
                delay_s: float = 1.0) -> T:
    """Call ``fn`` every ``delay_s`` until ``done(result)``; raise RetryTimeout after ``timeout_s``."""
    deadline = time.monotonic() + timeout_s
    while True:
        r = fn()
        if done(r):
            return r
        if time.monotonic() >= deadline:
            raise RetryTimeout(f"condition not met within {timeout_s}s (last result {r!r})")
        time.sleep(delay_s)


def backoff_delays(start_s: float = 0.2, cap_s: float = 5.0, jitter: float = 0.1):
    d = start_s
    while True:
        yield d * (1 + random.uniform(-jitter, jitter))
        d = min(cap_s, d * 2)


def exec_with_backoff(fn: Callable[[], T], max_attempts: int = 10, start_s: float = 0.2, cap_s: float = 5.0,
                      retry_on: Tuple[Type[BaseException], ...] = (Exception,),
                      should_retry: Optional[Callable[[BaseException], bool]] = None) -> T:
    delays = backoff_delays(start_s, cap_s)
    last: Optional[BaseException] = None
    for attempt in range(max_attempts):
        try:
            return fn()
        except retry_on as e:  # noqa: PERF203
            if should_retry is not None and not should_retry(e):
                raise
            last = e
            if attempt + 1 < max_attempts:
                time.sleep(next(delays))
    assert last is not None
    raise last


def retry_on_errors(fn: Callable[[], T], max_attempts: int = 10, start_s: float = 0.2, cap_s: float = 5.0,
                    retry_on: Tuple[Type[BaseException], ...] = (Exception,)) -> T:
    return exec_with_backoff(fn, max_attempts, start_s, cap_s, retry_on)
