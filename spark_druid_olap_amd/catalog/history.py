"""Bounded history of executed Druid queries.

Parity: ``sd/metadata/DruidQueryHistory.scala:25-76`` (FIFO, default 500 entries, system property
``sparkline.queryhistory.maxsize``) and the ``DruidQueryExecutionView`` record (stage, partition,
server, segments, start, druidExecTime, queryExecTime, numRows, query JSON, SQL text).  Enabled by
``spark.sparklinedata.enable.druid.query.history``; exposed as the ``d$druidqueries`` view.
"""
from __future__ import annotations

import collections
import json
import os
import threading
import time
from dataclasses import asdict, dataclass
from typing import Deque, List, Optional


@dataclass
class DruidQueryExecutionView:
    queryId: str
    stageId: int
    partitionId: int
    taskAttemptId: int
    druidQueryServer: str
    druidSegIntervals: Optional[str]
    startTime: str
    druidExecTime: float
    queryExecTime: float
    numRows: int
    druidQuery: str
    sqlStmt: Optional[str] = None


class DruidQueryHistory:
    def __init__(self, max_size: Optional[int] = None):
        self.max_size = int(max_size or os.environ.get("sparkline.queryhistory.maxsize", 500))
        self._q: Deque[DruidQueryExecutionView] = collections.deque(maxlen=self.max_size)
        self._lock = threading.Lock()
        self._n = 0

    def add(self, view: DruidQueryExecutionView) -> None:
        with self._lock:
            self._q.append(view)
            self._n += 1

    def record(self, spec, exec_ms: float, total_ms: float, rows: int, server: str,
               sql: Optional[str] = None, segments: Optional[int] = None) -> DruidQueryExecutionView:
        with self._lock:
            self._n += 1
            qid = f"q{self._n}"
        v = DruidQueryExecutionView(
            queryId=qid, stageId=0, partitionId=0, taskAttemptId=0, druidQueryServer=server,
            druidSegIntervals=None if segments is None else f"{segments} segments",
            startTime=time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime()), druidExecTime=round(exec_ms, 3),
            queryExecTime=round(total_ms, 3), numRows=rows, druidQuery=json.dumps(spec.to_json()), sqlStmt=sql)
        with self._lock:
            self._q.append(v)
        return v

    def entries(self) -> List[DruidQueryExecutionView]:
        with self._lock:
            return list(self._q)

    def clear(self) -> None:
        with self._lock:
            self._q.clear()

    def rows(self) -> List[dict]:
        return [asdict(v) for v in self.entries()]
