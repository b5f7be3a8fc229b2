"""Drive every GPU rank from one client-facing server (the reference's HiveThriftServer2 fronts the
whole Spark + Druid cluster, ``asql/hive/thriftserver/sparklinedata/HiveThriftServer2.scala:55-79``).

Each rank holds a shard of every datasource, so every statement must run on every rank, in the same
order (the merges inside a query are collectives).  Rank 0 accepts the client connections; its
``SpmdDispatcher`` serialises statements from all client sessions into one stream and broadcasts
each one -- with the client session's id, ``SET`` overlay and a deadline -- to the other ranks
(``World.broadcast_object``).  Every rank then executes it over its own shard and the collectives
inside merge the partial aggregates; rank 0 returns the (global) result to the client.  The other
ranks run ``serve_peer``: a loop that receives and executes the same stream, keeping a mirror of
every client session (conf + current database) so session state evolves identically everywhere.

Identical statements from different clients that queue up together execute once (a shared scan;
``engine/scheduler.py`` explains the rule).  While idle the dispatcher broadcasts a heartbeat, so
peers never sit in a collective longer than the process-group timeout.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

log = logging.getLogger("sdo.spmd")

HEARTBEAT_S = 20.0


class _Item:
    __slots__ = ("msg", "event", "result", "error")

    def __init__(self, msg: Dict[str, Any]):
        self.msg = msg
        self.event = threading.Event()
        self.result = None
        self.error: Optional[BaseException] = None


def _execute(sessions: Dict[bytes, Any], root, msg: Dict[str, Any]):
    """Apply one broadcast message to this rank's session mirrors; returns a pandas frame for
    statements (None for session lifecycle messages)."""
    op = msg["op"]
    sid = msg.get("sid")
    if op == "open":
        s = root.new_session()
        for k, v in (msg.get("conf") or {}).items():
            s.conf.set(k, v)
        if msg.get("db"):
            s.catalog.use(msg["db"])
        sessions[sid] = s
        return None
    if op == "close":
        sessions.pop(sid, None)
        return None
    if op == "exec":
        s = sessions.get(sid)
        if s is None:
            s = sessions[sid] = root.new_session()
        for k, v in (msg.get("overlay") or {}).items():
            s.conf.set(k, v)
        token = None
        if msg.get("timeout_s"):
            from ..utils.cancel import CancelToken

            token = CancelToken(float(msg["timeout_s"]) * 1000.0)
        df = s.sql(msg["stmt"])
        return df, df.to_pandas(token=token)
    return None


class SpmdDispatcher:
    """Rank 0 side: one ordered statement stream for every rank."""

    def __init__(self, session, world):
        self.root = session
        self.world = world
        self.sessions: Dict[bytes, Any] = {}
        self._q: "queue.Queue[_Item]" = queue.Queue()
        self._stop = threading.Event()
        self.stats = {"statements": 0, "executions": 0, "coalesced": 0, "heartbeats": 0}
        self._thread = threading.Thread(target=self._loop, daemon=True, name="spmd-dispatch")
        self._thread.start()

    # ---------------------------------------------------------------- client-facing API (rank 0)
    def open_session(self, sid: bytes, conf: Dict[str, str], db: Optional[str]) -> None:
        self._submit({"op": "open", "sid": sid, "conf": dict(conf), "db": db})

    def close_session(self, sid: bytes) -> None:
        self._submit({"op": "close", "sid": sid})

    def session(self, sid: bytes):
        return self.sessions.get(sid)

    def execute(self, sid: bytes, stmt: str, overlay: Optional[Dict[str, str]] = None,
                timeout_s: Optional[float] = None) -> Tuple[Any, Any]:
        """Run ``stmt`` for client session ``sid`` on every rank; returns (DataFrame, pandas)."""
        return self._submit({"op": "exec", "sid": sid, "stmt": stmt, "overlay": dict(overlay or {}),
                             "timeout_s": timeout_s})

    def shutdown(self) -> None:
        if not self._stop.is_set():
            self._stop.set()
            self._thread.join(timeout=HEARTBEAT_S + 5)

    def _submit(self, msg):
        it = _Item(msg)
        self._q.put(it)
        it.event.wait()
        if it.error is not None:
            raise it.error
        return it.result

    # ---------------------------------------------------------------- dispatch loop
    def _loop(self):
        w = self.world
        while True:
            try:
                first = self._q.get(timeout=HEARTBEAT_S)
            except queue.Empty:
                if self._stop.is_set():
                    break
                try:
                    w.broadcast_object({"op": "noop"})
                except BaseException as e:  # noqa: BLE001
                    if not _elastic_recover(self.root, e):
                        raise
                    w = self.world = self.root.engine.world
                self.stats["heartbeats"] += 1
                continue
            batch = [first]
            while True:  # everything queued right now travels in one broadcast
                try:
                    batch.append(self._q.get_nowait())
                except queue.Empty:
                    break
            groups = self._coalesce(batch)
            msgs = [g[0].msg for g in groups]
            try:
                w.broadcast_object({"op": "batch", "msgs": msgs})
            except BaseException as e:  # noqa: BLE001
                if _elastic_recover(self.root, e):  # a peer is gone: rebuild, then serve again
                    w = self.world = self.root.engine.world
                    for it in batch:
                        self._q.put(it)
                    continue
                for it in batch:
                    it.error = e
                    it.event.set()
                raise
            for g in groups:
                try:
                    res = _run_elastic(self.root, lambda m=g[0].msg: _execute(self.sessions, self.root, m))
                    w = self.world = self.root.engine.world
                    for it in g:
                        it.result = res
                except BaseException as e:  # noqa: BLE001  (every rank raised the same way)
                    for it in g:
                        it.error = e
                for it in g:
                    it.event.set()
            if self._stop.is_set() and self._q.empty():
                break
        w.broadcast_object({"op": "stop"})

    def _coalesce(self, batch: List[_Item]) -> List[List[_Item]]:
        """Group identical read-only statements of sessions in the same state (same conf and
        current database): they execute once."""
        out: List[List[_Item]] = []
        index: Dict[Any, int] = {}
        for it in batch:
            m = it.msg
            key = None
            if m["op"] == "exec" and not m.get("overlay") and _is_query(m["stmt"]):
                s = self.sessions.get(m["sid"])
                if s is not None and not s.catalog.temp:
                    key = (m["stmt"].strip(), s.catalog.current_db, tuple(sorted(s.conf.items().items())))
            if key is not None and key in index:
                out[index[key]].append(it)
                self.stats["coalesced"] += 1
                continue
            if key is not None:
                index[key] = len(out)
            out.append([it])
            if m["op"] == "exec":
                self.stats["statements"] += 1
        self.stats["executions"] += len(out)
        return out


def _is_query(stmt: str) -> bool:
    head = stmt.lstrip().lstrip("(").split(None, 1)[0].lower() if stmt.strip() else ""
    return head in ("select", "with")


def _elastic_recover(session, e: BaseException) -> bool:
    """Elastic mode (parallel/recovery.py enabled): a collective failed because a rank is gone --
    agree, rebuild the communicator over the survivors and re-home the lost shards."""
    from ..parallel import recovery

    if not recovery.is_comm_failure(e):
        return False
    log.warning("SPMD stream: collective failed (%s), recovering", e)
    recovery.recover(session)
    return True


def _run_elastic(session, fn):
    from ..parallel import recovery

    if recovery.state() is None:
        return fn()
    return recovery.run_with_recovery(session, fn)


def serve_peer(session, world) -> None:
    """Ranks 1..N-1: execute the statement stream broadcast by rank 0 until it stops."""
    sessions: Dict[bytes, Any] = {}
    while True:
        try:
            msg = world.broadcast_object(None)
        except BaseException as e:  # noqa: BLE001
            if not _elastic_recover(session, e):
                raise
            world = session.engine.world
            continue
        op = msg.get("op")
        if op == "stop":
            return
        if op == "noop":
            continue
        for m in msg.get("msgs", []):
            try:
                _run_elastic(session, lambda m=m: _execute(sessions, session, m))
                world = session.engine.world
            except BaseException as e:  # noqa: BLE001  (rank 0 reports the error to the client)
                log.debug("peer statement failed: %s", e)
