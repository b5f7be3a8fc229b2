"""Failure detection, agreement and fault injection for the multi-GPU query path.

The reference relies on ZooKeeper membership + HTTP errors + Spark task retry
(``sd/client/CuratorConnection.scala:77-133``, ``sd/DruidRDD.scala:428-493``); query execution
itself has no retry.  Across GPUs the hazard is different: if one rank fails its local
scan (a kernel error, an allocation failure, a cancelled token) and simply raises, its peers block
in the next collective until the process-group timeout.  So every rank reports a status word
*inside the collective it was going to issue anyway* (the one-shot all-gather buffer or the
variable-length count exchange, ``parallel/merge.py``): all ranks learn about the failure in the
same collective, raise consistently, and the process group stays in lock-step for the next query.

Fault injection (test-only) makes a chosen rank fail at a chosen point:
``SDO_FAULT_INJECT="rank=1,point=scan,times=1"`` or ``FaultInjector.configure(...)``.
Collective hangs (a rank that died outright) surface through the process-group timeout
(``SDO_COLLECTIVE_TIMEOUT_S``, default 600 s, ``parallel/world.py:init_world``).
"""
from __future__ import annotations

import os
import threading
from typing import Optional

from ..utils.errors import DruidDataSourceException

STATUS_OK = 0
STATUS_FAILED = 1
STATUS_P2P_TIMEOUT = 3   # a peer never finished a peer-to-peer merge epoch (ops/csrc/p2p.h)
STATUS_P2P_RETRY = 4     # a P2P merge epoch was abandoned by every rank: re-run it over RCCL


class InjectedFault(DruidDataSourceException):
    """The fault injector failed this rank on purpose."""


class RankFailure(DruidDataSourceException):
    """Another rank failed its part of the query; every rank aborts the query consistently."""


class P2PRetry(RankFailure):
    """Every rank abandoned a peer-to-peer merge epoch together (a soft wait expired somewhere):
    the statement is re-run with the merge over RCCL (parallel/p2p.py, engine/executor.py)."""


class FaultInjector:
    def __init__(self):
        self._lock = threading.Lock()
        self.rank: Optional[int] = None
        self.point: Optional[str] = None
        self.times = 0
        spec = os.environ.get("SDO_FAULT_INJECT")
        if spec:
            kv = dict(x.split("=", 1) for x in spec.split(",") if "=" in x)
            self.configure(int(kv.get("rank", 0)), kv.get("point", "scan"), int(kv.get("times", 1)))

    def configure(self, rank: Optional[int], point: Optional[str] = "scan", times: int = 1) -> None:
        with self._lock:
            self.rank, self.point, self.times = rank, point, int(times)

    def clear(self) -> None:
        self.configure(None, None, 0)

    def maybe_fail(self, point: str, rank: int) -> None:
        with self._lock:
            if self.times <= 0 or self.point != point or self.rank != rank:
                return
            self.times -= 1
        raise InjectedFault(f"injected fault at {point} on rank {rank}")


FAULTS = FaultInjector()


def raise_if_failed(statuses, my_rank: int, local_error: Optional[BaseException]) -> None:
    """After the status exchange: the failing rank re-raises its own error, the others raise
    RankFailure naming the failed ranks."""
    bad = [r for r, s in enumerate(statuses) if int(s) != STATUS_OK]
    if local_error is not None:
        raise local_error
    if bad and all(int(statuses[r]) == STATUS_P2P_RETRY for r in bad):
        raise P2PRetry("peer-to-peer merge epoch abandoned by every rank: retrying over RCCL")
    if bad:
        what = "timed out in a peer-to-peer merge" if any(int(statuses[r]) == STATUS_P2P_TIMEOUT for r in bad) \
            else "failed their local scan"
        raise RankFailure(f"query aborted: rank(s) {bad} {what}")
