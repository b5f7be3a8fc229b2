"""Drive every GPU rank from one client-facing server (the reference's HiveThriftServer2 fronts the
whole Spark + Druid cluster, ``asql/hive/thriftserver/sparklinedata/HiveThriftServer2.scala:55-79``).

Each rank holds a shard of every datasource, so every statement must run on every rank (the merges
inside a query are collectives).  Rank 0 accepts the client connections; its ``SpmdDispatcher``
orders the statements of all client sessions into one stream and broadcasts it -- with the client
session's id, ``SET`` overlay and a deadline -- to the other ranks (``World.broadcast_object``).
The other ranks run ``serve_peer``: they receive and apply the same stream, keeping a mirror of
every client session (conf + current database) so session state evolves identically everywhere.

Concurrency across all GPUs.  The reference serves many BI clients against the whole cluster at
once (pooled HTTP client 100/20, ``asd/DruidPlanner.scala:83-90``; a JMeter fair-pool load,
``docs/bi-benchmark/snap-sales-demo.jmx:87-101``).  Here every rank runs K *execution slots*: one
worker thread per slot, each with its own process group (``dist.new_group``, created in the same
order on every rank), its own HIP stream and its own device buffers.  Rank 0 assigns each query to
a slot and the assignment travels in the broadcast, so within a slot every rank runs the same
statements in the same order -- its collectives match -- while statements of different slots run
at the same time on independent communicators.  Everything that may issue collectives outside a
statement's own slot -- planning and lowering (cluster-wide FD tables, row estimates), commands,
plans whose pushed queries are re-planned at run time (subquery-parameterised filters, fused
grouping sets) -- runs in the dispatch thread, in broadcast order, on the default group.

Identical statements from different clients that queue up together may execute once (a shared
scan; ``engine/scheduler.py`` explains the rule; ``SDO_SPMD_COALESCE=0`` turns it off).  While idle
the dispatcher broadcasts a heartbeat, so peers never sit in a collective longer than the
process-group timeout.
"""
from __future__ import annotations

import logging
import os
import queue
import threading
from typing import Any, Dict, List, Optional, Tuple

from ..parallel.world import statement_turn

log = logging.getLogger("sdo.spmd")

HEARTBEAT_S = 20.0
INLINE = -1  # slot id of statements that run in the dispatch thread


class _Item:
    __slots__ = ("msg", "event", "result", "error")

    def __init__(self, msg: Dict[str, Any]):
        self.msg = msg
        self.event = threading.Event()
        self.result = None
        self.error: Optional[BaseException] = None


def _session_for(sessions: Dict[bytes, Any], root, msg: Dict[str, Any]):
    sid = msg.get("sid")
    s = sessions.get(sid)
    if s is None:
        s = sessions[sid] = root.new_session()
    for k, v in (msg.get("overlay") or {}).items():
        s.conf.set(k, v)
    return s


def _apply(sessions: Dict[bytes, Any], root, msg: Dict[str, Any]) -> None:
    """Session lifecycle messages (every rank, dispatch thread, broadcast order)."""
    op = msg["op"]
    sid = msg.get("sid")
    if op == "open":
        s = root.new_session()
        for k, v in (msg.get("conf") or {}).items():
            s.conf.set(k, v)
        if msg.get("db"):
            s.catalog.use(msg["db"])
        sessions[sid] = s
    elif op == "close":
        sessions.pop(sid, None)
        # a client that closes its session without closing its cursors: release them (every rank
        # applies the close in broadcast order, so every rank drops the same iterators)
        for k in [k for k, owner in _STREAM_OWNER.items() if owner == sid]:
            _STREAMS.pop(k, None)
            _STREAM_OWNER.pop(k, None)


def _token(msg):
    if msg.get("timeout_s"):
        from ..utils.cancel import CancelToken

        return CancelToken(float(msg["timeout_s"]) * 1000.0)
    return None


def _run_statement(df, msg):
    """Execute a planned statement; rank 0 answers the client, so the final groups of its pushed
    queries gather there only (engine/executor.py results_on_root)."""
    from ..engine.executor import results_on_root

    with results_on_root():
        return df, df.to_pandas(token=_token(msg))


# Open Select cursors of streamed statements on this rank (stream id -> page iterator).  Every
# rank advances a cursor on the same broadcast message, so the page's collectives (the Select
# page gather) run in lock step; rank 0 hands the page to the client.
_STREAMS: Dict[int, Any] = {}
_STREAM_OWNER: Dict[int, Any] = {}  # stream id -> client session id (released with the session)


def _streamable(df, s) -> bool:
    """A Select-backed or large groupBy statement (every rank decides alike: the groupBy check
    prepares the pushed query, in broadcast order)."""
    return df.plan is not None and bool(s.conf.typed("spark.sparklinedata.druid.stream.results")) and \
        (df._stream_source()[1] is not None or df.agg_streamable())


def _execute(sessions: Dict[bytes, Any], root, msg: Dict[str, Any]):
    """Apply one message in the dispatch thread: lifecycle ops, commands, statements that do not
    run on a slot and Select cursor steps.  Returns (DataFrame, pandas) for statements --
    (DataFrame, ("stream", id)) for a streamed Select -- a page for a cursor step, else None."""
    op = msg["op"]
    if op == "stream_next":
        it = _STREAMS.get(msg["stream_id"])
        page = next(it, None) if it is not None else None
        if page is None:
            _STREAMS.pop(msg["stream_id"], None)
            _STREAM_OWNER.pop(msg["stream_id"], None)
        return page
    if op == "stream_close":
        _STREAMS.pop(msg["stream_id"], None)
        _STREAM_OWNER.pop(msg["stream_id"], None)
        return None
    if op != "exec":
        _apply(sessions, root, msg)
        return None
    s = _session_for(sessions, root, msg)
    df = s.sql(msg["stmt"])  # (commands -- CREATE TABLE AS SELECT -- run here, on every rank)
    if msg.get("stream_id") is not None and _streamable(df, s):
        # a Select-backed result pages through the cursor instead of materialising (the
        # reference's DruidSelectResultIterator); the first page runs on the first step
        _STREAMS[msg["stream_id"]] = df.iter_batches(token=_token(msg))
        _STREAM_OWNER[msg["stream_id"]] = msg.get("sid")
        return df, ("stream", msg["stream_id"])
    return _run_statement(df, msg)


def slot_eligible(df) -> bool:
    """A planned statement may run on a slot when nothing it executes issues collectives outside
    its own slot: a query plan whose pushed queries are all known (and so prepared) up front."""
    from ..query import spec as S
    from ..sql import plan as P

    if df.plan is None:
        return False
    if P.find_all(df.plan, P.Union):   # fused grouping sets prepare their scan at run time
        return False
    dqs = P.find_all_deep(df.plan, P.DruidQuery)
    return not any(S.find_deferred(dq.spec) for dq in dqs)


def prepare_statement(sessions: Dict[bytes, Any], root, msg: Dict[str, Any]):
    """Plan the statement and lower every pushed query (dispatch thread, broadcast order: the
    collectives of lowering run on the default group identically on every rank)."""
    from ..sql import plan as P

    s = _session_for(sessions, root, msg)
    df = s.sql(msg["stmt"])
    for dq in P.find_all_deep(df.plan, P.DruidQuery):
        s.prepare_druid(dq)
    return df


class SlotWorkers:
    """K execution slots on this rank: a worker thread each, with its own process group (created
    collectively, same order on every rank), HIP stream and device-buffer slot."""

    BUFFER_SLOT_BASE = 100  # engine/scheduler.py buffer slots (1..K belong to the local scheduler)

    def __init__(self, session, world, k: int):
        import torch
        import torch.distributed as dist

        from ..parallel.world import IssueOrder

        self.k = k
        self.groups = [dist.new_group(list(range(world.size))) if world.distributed else None for _ in range(k)]
        # the control stream (statement broadcasts, heartbeats) over a host-side gloo group of the
        # same ranks: under RCCL a control broadcast would otherwise sit in a GPU queue next to the
        # slots' collectives, in an order that differs per rank
        self.ctrl = dist.new_group(list(range(world.size)), backend="gloo") \
            if world.distributed and world.backend == "nccl" else None
        self.world = world
        # every statement's sequence number, in broadcast order: the slots' collectives leave this
        # rank in that order (parallel/world.py IssueOrder -- no cross-communicator deadlock)
        self.order = IssueOrder() if world.distributed else None
        dev = world.device()
        self.streams = [torch.cuda.Stream(dev) if dev.type == "cuda" else None for _ in range(k)]
        self.queues: List["queue.Queue"] = [queue.Queue() for _ in range(k)]
        self.busy = [0] * k
        self.max_inflight = 0
        self._lock = threading.Lock()
        self.threads = [threading.Thread(target=self._work, args=(i,), daemon=True, name=f"spmd-slot-{i}")
                        for i in range(k)]
        for t in self.threads:
            t.start()

    def submit(self, slot: int, df, msg, done) -> None:
        with self._lock:
            self.busy[slot] += 1
        self.queues[slot].put((df, msg, done))

    def control(self, world):
        """The group control broadcasts use (None: the world's own) -- only while ``world`` is the
        one the slots were built for (an elastic recovery replaces it)."""
        return self.ctrl if world is self.world else None

    def least_busy(self) -> int:
        with self._lock:
            return min(range(self.k), key=lambda i: self.busy[i])

    def stop(self) -> None:
        for q in self.queues:
            q.put(None)
        for t in self.threads:
            t.join(timeout=5)

    def _work(self, i: int) -> None:
        import torch

        from ..engine.scheduler import use_slot
        from ..parallel.world import slot_group

        while True:
            job = self.queues[i].get()
            if job is None:
                return
            df, msg, done = job
            res, err = None, None
            with self._lock:
                self.max_inflight = max(self.max_inflight, sum(1 for b in self.busy if b > 0))
            try:
                with statement_turn(self.order, msg.get("seq")), slot_group(self.groups[i]), \
                        use_slot(self.BUFFER_SLOT_BASE + i):
                    if self.streams[i] is not None:
                        # preparation (dispatch thread, default stream) launched device work the
                        # scan reads -- e.g. the u16 HLL code planes of segment/hllcode.py
                        self.streams[i].wait_stream(torch.cuda.default_stream(self.streams[i].device))
                        with torch.cuda.stream(self.streams[i]):
                            res = _run_statement(df, msg)
                        self.streams[i].synchronize()
                    else:
                        res = _run_statement(df, msg)
            except BaseException as e:  # noqa: BLE001  (rank 0 reports it; peers drop it)
                err = e
            finally:
                with self._lock:
                    self.busy[i] -= 1
            done(res, err)


class SpmdDispatcher:
    """Rank 0 side: one ordered statement stream for every rank, executed on K slots."""

    def __init__(self, session, world, slots: Optional[int] = None, coalesce: Optional[bool] = None):
        self.root = session
        self.world = world
        self.sessions: Dict[bytes, Any] = {}
        self._q: "queue.Queue[_Item]" = queue.Queue()
        self._stop = threading.Event()
        self.coalesce = coalesce if coalesce is not None else os.environ.get("SDO_SPMD_COALESCE", "1") != "0"
        k = slots if slots is not None else int(os.environ.get("SDO_SPMD_SLOTS", "4"))
        if world.distributed:
            world.broadcast_object({"op": "slots", "k": k})  # peers create the same slot groups
        self.workers = SlotWorkers(session, world, k) if k > 0 else None
        self._pinned: Dict[bytes, int] = {}
        self._sid_lock = threading.Lock()
        self._stream_seq = 0
        self.stats = {"statements": 0, "executions": 0, "coalesced": 0, "heartbeats": 0, "on_slots": 0,
                      "inline": 0}
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
                timeout_s: Optional[float] = None, stream: bool = False) -> Tuple[Any, Any]:
        """Run ``stmt`` for client session ``sid`` on every rank; returns (DataFrame, pandas).  With
        ``stream`` a Select-backed statement returns (DataFrame, ("stream", id)) instead: pull its
        pages with ``stream_next(id)``, release it with ``close_stream(id)``."""
        msg = {"op": "exec", "sid": sid, "stmt": stmt, "overlay": dict(overlay or {}), "timeout_s": timeout_s}
        if stream:
            with self._sid_lock:
                self._stream_seq += 1
                msg["stream_id"] = self._stream_seq
        return self._submit(msg)

    def stream_next(self, stream_id: int):
        """The next page (pandas) of a streamed statement on every rank; None at the end."""
        return self._submit({"op": "stream_next", "stream_id": stream_id})

    def close_stream(self, stream_id: int) -> None:
        self._submit({"op": "stream_close", "stream_id": stream_id})

    def shutdown(self) -> None:
        if not self._stop.is_set():
            self._stop.set()
            self._thread.join(timeout=HEARTBEAT_S + 5)
        if self.workers is not None:
            self.workers.stop()

    def _submit(self, msg):
        it = _Item(msg)
        self._q.put(it)
        it.event.wait()
        if it.error is not None:
            raise it.error
        return it.result

    # ---------------------------------------------------------------- dispatch loop
    def _assign(self, groups: List[List[_Item]]) -> List[int]:
        """Slot per group of identical statements: queries whose plans allow it go to a slot, the
        rest (commands, session ops, run-time re-planned queries) run inline."""
        out = []
        for g in groups:
            m = g[0].msg
            slot = INLINE
            if self.workers is not None and m["op"] == "exec" and _is_query(m["stmt"]) and not m.get("overlay") \
                    and not _plans_collectively(m["stmt"]):
                try:
                    s = _session_for(self.sessions, self.root, {"sid": m["sid"]})
                    df = s.sql(m["stmt"])
                    streamed = m.get("stream_id") is not None and _streamable(df, s)  # cursors run inline
                    if slot_eligible(df) and not streamed:
                        slot = self._session_slot(m["sid"])
                except Exception:  # noqa: BLE001  (the statement fails the same way inline)
                    slot = INLINE
            out.append(slot)
        return out

    def _session_slot(self, sid) -> int:
        """A session with work still queued keeps its slot (its statements stay in order); else the
        least busy slot."""
        s = self._pinned.get(sid)
        if s is not None and self.workers.busy[s] > 0:
            return s
        s = self._pinned[sid] = self.workers.least_busy()
        return s

    def _loop(self):
        w = self.world
        while True:
            try:
                first = self._q.get(timeout=HEARTBEAT_S)
            except queue.Empty:
                if self._stop.is_set():
                    break
                try:
                    w.broadcast_object({"op": "noop"}, group=self._ctrl(w))
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
            slots = self._assign(groups)
            msgs = [dict(g[0].msg, slot=sl) for g, sl in zip(groups, slots)]
            order = self._order()
            if order is not None:
                for m in msgs:
                    m["seq"] = order.begin()
            try:
                w.broadcast_object({"op": "batch", "msgs": msgs}, group=self._ctrl(w))
            except BaseException as e:  # noqa: BLE001
                if order is not None:
                    for m in msgs:
                        order.finish(m["seq"])
                if _elastic_recover(self.root, e):  # a peer is gone: rebuild, then serve again
                    w = self.world = self.root.engine.world
                    for it in batch:
                        self._q.put(it)
                    continue
                for it in batch:
                    it.error = e
                    it.event.set()
                raise
            for g, m in zip(groups, msgs):
                if m["slot"] != INLINE:
                    self.stats["on_slots"] += 1
                    self._dispatch_slot(g, m)
                    continue
                self.stats["inline"] += 1
                try:
                    with statement_turn(order, m.get("seq")):
                        res = _run_elastic(self.root, lambda m=m: _execute(self.sessions, self.root, m))
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
        w.broadcast_object({"op": "stop"}, group=self._ctrl(w))

    def _ctrl(self, w):
        return self.workers.control(w) if self.workers is not None else None

    def _order(self):
        return self.workers.order if self.workers is not None else None

    def _dispatch_slot(self, g: List[_Item], m: Dict[str, Any]) -> None:
        try:
            with statement_turn(self._order(), m.get("seq"), finish=False):
                df = prepare_statement(self.sessions, self.root, m)
        except BaseException as e:  # noqa: BLE001
            if self._order() is not None:
                self._order().finish(m["seq"])
            for it in g:
                it.error = e
                it.event.set()
            return

        def done(res, err, g=g):
            for it in g:
                it.result, it.error = res, err
                it.event.set()
        self.workers.submit(m["slot"], df, m, done)

    def _coalesce(self, batch: List[_Item]) -> List[List[_Item]]:
        """Group identical read-only statements of sessions in the same state (same conf and
        current database): they execute once."""
        out: List[List[_Item]] = []
        index: Dict[Any, int] = {}
        for it in batch:
            m = it.msg
            key = None
            if self.coalesce and m["op"] == "exec" and not m.get("overlay") and _is_query(m["stmt"]) and \
                    m.get("stream_id") is None:  # (a cursor belongs to one client)
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


def _plans_collectively(stmt: str) -> bool:
    """Statements whose *planning* issues collectives: the ``d$*`` metadata views gather the
    cluster-wide inventory from every rank when analysed (catalog/views.py cluster_inventory).  Rank
    0 must not plan them alone while deciding a slot (its peers sit in the broadcast): they run
    inline, planned once, in broadcast order on every rank."""
    return "d$" in stmt.lower()


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
    workers: Optional[SlotWorkers] = None
    while True:
        try:
            msg = world.broadcast_object(None, group=workers.control(world) if workers is not None else None)
        except BaseException as e:  # noqa: BLE001
            if not _elastic_recover(session, e):
                raise
            world = session.engine.world
            continue
        op = msg.get("op")
        if op == "stop":
            if workers is not None:
                workers.stop()
            return
        if op == "noop":
            continue
        if op == "slots":
            k = int(msg["k"])
            workers = SlotWorkers(session, world, k) if k > 0 else None
            continue
        order = workers.order if workers is not None else None
        for m in msg.get("msgs", []):
            if order is not None and m.get("seq") is not None:
                order.begin(m["seq"])
        for m in msg.get("msgs", []):
            slot = m.get("slot", INLINE)
            submitted = False
            try:
                if slot != INLINE and workers is not None:
                    with statement_turn(order, m.get("seq"), finish=False):
                        df = prepare_statement(sessions, session, m)
                    workers.submit(slot, df, m, lambda res, err: None)  # rank 0 answers the client
                    submitted = True
                    continue
                with statement_turn(order, m.get("seq")):
                    _run_elastic(session, lambda m=m: _execute(sessions, session, m))
                world = session.engine.world
            except BaseException as e:  # noqa: BLE001  (rank 0 reports the error to the client)
                log.debug("peer statement failed: %s", e)
            finally:
                if order is not None and m.get("seq") is not None and slot != INLINE and not submitted:
                    order.finish(m["seq"])
