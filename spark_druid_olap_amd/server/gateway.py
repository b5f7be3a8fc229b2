"""HiveServer2 endpoint with the native gateway (``server/csrc/hs2_gateway.cpp``) in front.

``NativeHiveServer`` is a ``HiveThriftServer`` whose connections are served by the C++ gateway:
per-statement work (socket I/O, SASL, Thrift decoding/encoding, identical-statement batching,
status polls and result paging) never takes the GIL.  What remains in Python scales with the number
of *executions*:

* ``K`` executor threads pull batches from the gateway (``next_batch`` waits with the GIL released),
  run the statement on the leader's session inside a HIP-stream slot lease (engine/scheduler.py) --
  or through the SPMD dispatcher when several ranks serve (server/spmd.py) -- and hand the typed
  columns back once (``finish_batch``); the gateway slices pages for every attached operation;
* every RPC the gateway does not handle natively (OpenSession / CloseSession, commands such as
  SET / USE / CREATE, metadata calls, statements with a confOverlay or a timeout, operations the
  Python side owns) arrives here as raw message bytes and runs through the inherited ``rpc_*``
  methods;
* after anything that can change a session's planning context (open, SET, USE, temp views) the
  session's context token is re-published, so only statements that would plan identically batch.

The pure-Python server stays available (``SDO_NATIVE_GATEWAY=0`` or when the extension is absent on
a CPU-only checkout) and is the reference the native one is tested against (tests/test_gateway.py).
"""
from __future__ import annotations

import functools
import importlib
import json
import logging
import os
import threading
import time
from typing import List, Optional, Tuple

import torch

import numpy as np
import pandas as pd

from . import thrift as T
from .hive_server import HiveThriftServer, Operation

log = logging.getLogger("sdo.gateway")


def load_native():
    """The compiled gateway module (built in-tree by ops/build.py:build_gateway).  ``SDO_GATEWAY_SO``
    names an alternative build of the same module (the host ASan/UBSan build of tools/asan_host.py)."""
    alt = os.environ.get("SDO_GATEWAY_SO")
    if alt:
        import sys
        from importlib import util as _ilu

        name = "spark_druid_olap_amd.server._sdo_gateway"
        if name not in sys.modules:
            spec = _ilu.spec_from_file_location(name, alt)
            mod = _ilu.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules[name] = mod
        return sys.modules[name]
    try:
        return importlib.import_module("spark_druid_olap_amd.server._sdo_gateway")
    except ImportError:
        from ..ops import build as B

        B.build_gateway()
        return importlib.import_module("spark_druid_olap_amd.server._sdo_gateway")


def context_token(sess) -> int:
    """Everything per-session that changes how a statement plans (the plan cache key minus the
    statement text and the shared catalog state)."""
    cat = sess.catalog
    key = (cat.current_db, id(cat.temp) if cat.temp else 0, sess.conf.cache_key())
    return hash(key) & 0x7FFFFFFFFFFFFFFF


# column kinds understood by the gateway's TRowSet encoder
_KIND = {"boolean": (0, np.uint8), "tinyint": (1, np.int8), "smallint": (2, np.int16), "int": (3, np.int32),
         "bigint": (4, np.int64), "double": (5, np.float64), "float": (5, np.float64), "decimal": (5, np.float64)}


def result_columns(df) -> list:
    """The result's columns: Series of a pandas frame, or the SQL executor's Batch columns -- numeric
    ones as their numpy values (no DataFrame and no Series are built on the serving path)."""
    if isinstance(df, pd.DataFrame):
        return [df.iloc[:, i] for i in range(df.shape[1])]
    out = []
    for r in df.refs:
        a = df.cols.array(r.rid)
        out.append(a if a is not None else df.cols[r.rid])
    return out


def encode_columns(types: List[str], df) -> List[Tuple[int, bytes, bytes, bytes]]:
    """Typed columns for the gateway: (kind, little-endian values | utf-8 blob, int64 offsets for
    strings, one null byte per row).  Same value rendering as the Python server (_tcolumn).
    ``df``: a pandas frame, a list of Series, or the SQL executor's Batch."""
    out = []
    cols = df if isinstance(df, list) else result_columns(df)
    for t, s in zip(types, cols):
        base = t.split("(")[0]
        arr = s.to_numpy() if isinstance(s, pd.Series) else np.asarray(s)
        if arr.dtype.kind in "iub":
            isna = np.zeros(len(arr), dtype=bool)            # numpy ints / bools hold no nulls
        elif arr.dtype.kind == "f":
            isna = np.isnan(arr)
        else:
            isna = pd.isna(s).to_numpy(dtype=bool) if len(arr) else np.zeros(0, dtype=bool)
        nulls = isna.view(np.uint8).tobytes()
        if base in _KIND:
            kind, dt = _KIND[base]
            if base == "boolean":
                vals = np.array([bool(v) if not n else False for v, n in zip(arr.tolist(), isna)], dtype=np.uint8)
            elif arr.dtype.kind in "iufb":
                vals = np.where(isna, 0, arr) if isna.any() else arr
            else:
                num = pd.to_numeric(pd.Series(arr), errors="coerce")
                if kind == 5:
                    vals = num.to_numpy(dtype=np.float64, na_value=0.0)
                else:
                    vals = num.fillna(0).to_numpy().astype(dt)
            out.append((kind, np.ascontiguousarray(vals, dtype=dt).tobytes(), b"", nulls))
            continue
        s = pd.Series(arr) if not isinstance(s, pd.Series) else s
        vals = s.tolist()
        offs = np.zeros(len(vals) + 1, dtype=np.int64)
        if vals and not isna.any() and all(type(v) is str for v in vals):
            # plain strings (the common case): C-level join / len; byte lengths equal character
            # lengths when the text is ASCII (checked on the joined bytes)
            text = "".join(vals)
            blob = text.encode()
            if len(blob) == len(text):
                np.cumsum(np.fromiter(map(len, vals), dtype=np.int64, count=len(vals)), out=offs[1:])
                out.append((6, blob, offs.tobytes(), nulls))
                continue
        strs = []
        for v, n in zip(vals, isna):
            if n:
                strs.append(b"")
            elif isinstance(v, pd.Timestamp):
                strs.append((v.strftime("%Y-%m-%d") if base == "date" else str(v)).encode())
            else:
                strs.append(str(v).encode())
        np.cumsum(np.fromiter(map(len, strs), dtype=np.int64, count=len(strs)), out=offs[1:])
        out.append((6, b"".join(strs), offs.tobytes(), nulls))
    return out


def encode_schema(names: List[str], types: List[str]) -> bytes:
    """A complete TTableSchema struct (the gateway splices it into GetResultSetMetadata)."""
    return _encode_schema(tuple(names), tuple(types))


@functools.lru_cache(maxsize=4096)
def _encode_schema(names: Tuple[str, ...], types: Tuple[str, ...]) -> bytes:
    cols = []
    for i, (n, t) in enumerate(zip(names, types)):
        tid = T.TYPE_IDS.get(t.split("(")[0], T.TYPE_IDS["string"])
        cols.append({"columnName": n, "typeDesc": {"types": [{"primitiveEntry": {"type": tid}}]}, "position": i + 1})
    w = T.Writer()
    w.struct("TTableSchema", {"columns": cols})
    return bytes(w.buf)


class _BatchToken:
    """Cancellation for a batch: set once every operation attached to it was cancelled/closed."""

    def __init__(self, gw, bid):
        from ..utils.cancel import CancelToken

        self._gw, self._bid = gw, bid
        self._tok = CancelToken()
        self.deadline = None
        self.reason = "cancelled by client"

    @property
    def cancelled(self) -> bool:
        return self._gw.is_cancelled(self._bid)

    def cancel(self, reason: str = "cancelled") -> None:
        self._tok.cancel(reason)

    def check(self) -> None:
        from ..utils.errors import QueryCancelled

        if self._tok.cancelled or self._gw.is_cancelled(self._bid):
            raise QueryCancelled(self.reason)


class NativeHiveServer(HiveThriftServer):
    def __init__(self, session, host: str = "127.0.0.1", port: int = 10000, auth: str = "auto", world=None,
                 executors: Optional[int] = None):
        super().__init__(session, host, port, auth, world)
        self.nexec = executors or int(os.environ.get("SDO_GATEWAY_EXECUTORS", "0")) or \
            (session.engine.coalescer().scheduler.nslots + 2)
        self._gw = None
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        # per-statement timeline (tools/concurrency_bench.py --timeline): admission queue, prepare
        # (lowering / first-seen compile), slot wait, run (host + GPU, lease end synchronised),
        # encode -- a list of dicts while enabled, None otherwise
        self.timeline: Optional[list] = None
        # stall watchdog (with the timeline): when no execution has finished for STALL_S while some
        # are running, the Python stacks of the executor and compile threads -- where a device-wide
        # pause (allocator free-all, code-object load, a lock) holds every slot at once
        self.stalls: Optional[list] = None
        self._busy = 0
        self._busy_lock = threading.Lock()
        self._last_done = time.perf_counter()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "NativeHiveServer":
        from ..utils.memory import reserve_runtime_memory, serving_gc

        serving_gc()
        reserve_runtime_memory()  # device memory the HIP runtime allocates outside torch (scratch, RCCL)
        mod = load_native()
        self._gw = mod.Gateway(self.host, self.port, self._forward)
        # SDO_COALESCE=0: every statement executes (engine throughput, not result sharing)
        self._gw.set_coalesce(os.environ.get("SDO_COALESCE", "1") != "0")
        self.port = self._gw.start()
        for i in range(self.nexec):
            t = threading.Thread(target=self._executor, daemon=True, name=f"hs2-exec-{i}")
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._watchdog, daemon=True, name="hs2-stall-watchdog")
        t.start()
        self._threads.append(t)
        log.info("HiveServer2 endpoint (native gateway) on %s:%d, %d executors", self.host, self.port, self.nexec)
        return self

    def stop(self):
        self._stop.set()
        if self._gw is not None:
            self._gw.stop()
        for t in self._threads:
            t.join(5)
        if self.spmd is not None:
            self.spmd.shutdown()

    def stats(self) -> dict:
        return dict(self._gw.stats()) if self._gw is not None else {}

    def settle(self, timeout: float = 120.0) -> dict:
        """End of a warm-up (no statement running): wait for the background compiles the warm-up
        statements started, then size every slot's arena and partition scratch for the largest
        statement seen and return the allocator's leftover blocks to the device
        (engine/device_exec.py presize_device_memory).  The steady state then allocates nothing."""
        from ..engine.device_exec import presize_device_memory, wait_background_compiles

        waited = wait_background_compiles(timeout)
        sched = self.session.engine.coalescer().scheduler
        out = presize_device_memory(self.session.engine.world.device(), sched.nslots)
        out["compiles_waited"] = waited
        return out

    # ------------------------------------------------------------------ forwarded RPCs
    def _forward(self, msg: bytes) -> bytes:
        return self._dispatch(msg)

    def _publish(self, sid: bytes) -> None:
        ent = self.sessions.get(sid)
        if ent is not None and self._gw is not None:
            self._gw.set_context(sid, context_token(ent["session"]))

    def rpc_OpenSession(self, req):
        r = super().rpc_OpenSession(req)
        self._publish(r["sessionHandle"]["sessionId"]["guid"])
        return r

    def rpc_CloseSession(self, req):
        sid = req["sessionHandle"]["sessionId"]["guid"]
        if self._gw is not None:
            self._gw.drop_context(sid)
        return super().rpc_CloseSession(req)

    def _run(self, op: Operation, stmt: str, overlay):
        try:
            super()._run(op, stmt, overlay)
        finally:
            self._publish(op.session_id)  # SET / USE / CREATE TEMPORARY VIEW may have changed it

    # ------------------------------------------------------------------ batch executors
    @property
    def _metrics(self):
        from ..utils.metrics import metrics_of

        return metrics_of(self.session)

    def _executor(self):
        gw = self._gw
        while not self._stop.is_set():
            b = gw.next_batch(0.25)
            if b is None:
                continue
            bid, sid, stmt, queued_s = b
            t0 = time.perf_counter()
            tl = self.timeline
            rec = {"queue_ms": queued_s * 1e3} if tl is not None else None
            with self._busy_lock:
                self._busy += 1
            try:
                names, types, res = self._execute(bid, sid, stmt) if rec is None else \
                    self._execute(bid, sid, stmt, rec)
                t1 = time.perf_counter()
                self._metrics.record("gateway", (t1 - t0) * 1e3, True)
                schema = encode_schema(names, types)
                cols = encode_columns(types, res)
                gw.finish_batch(bid, schema, cols, res.n if hasattr(res, "n") else len(res), None)
                if rec is not None:
                    rec["encode_ms"] = (time.perf_counter() - t1) * 1e3
                    rec["t"] = t0
                    rec["stmt"] = stmt
                    tl.append(rec)
            except Exception as e:  # noqa: BLE001  (every attached operation reports it)
                self._metrics.record("gateway", (time.perf_counter() - t0) * 1e3, False)
                log.debug("batch %d failed: %s", bid, e)
                try:
                    gw.finish_batch(bid, b"", [], 0, f"{type(e).__name__}: {e}")
                except Exception:  # pragma: no cover
                    log.exception("finish_batch failed")
            finally:
                with self._busy_lock:
                    self._busy -= 1
                    self._last_done = time.perf_counter()

    STALL_S = 0.4

    def _watchdog(self):
        import sys
        import traceback

        armed = True
        while not self._stop.wait(0.02):
            st = self.stalls
            if st is None:
                continue
            idle = time.perf_counter() - self._last_done
            if self._busy <= 0 or idle < self.STALL_S:
                armed = True
                continue
            if not armed or len(st) >= 16:
                continue
            armed = False  # one capture per stall
            names = {t.ident: t.name for t in threading.enumerate()}
            stacks = {}
            for ident, fr in sys._current_frames().items():
                name = names.get(ident, "")
                if name.startswith(("hs2-exec", "sdo-jit")):
                    stacks[name] = [f"{os.path.basename(f.filename)}:{f.lineno} {f.name}"
                                    for f in traceback.extract_stack(fr)[-10:]]
            st.append({"t": time.perf_counter(), "idle_ms": round(idle * 1e3, 1), "busy": self._busy,
                       "stacks": stacks})

    def _execute(self, bid: int, sid: bytes, stmt: str, rec: Optional[dict] = None):
        ent = self.sessions.get(sid)
        if ent is None:
            raise RuntimeError("invalid session")
        token = _BatchToken(self._gw, bid)
        if self.spmd is not None:
            df, pdf = self.spmd.execute(sid, stmt, {}, None)
            return list(df.columns), [t for _, t in df.schema], pdf
        sess = ent["session"]
        ts = time.perf_counter()
        df = sess.sql(stmt)
        if rec is not None:
            rec["sql_ms"] = (time.perf_counter() - ts) * 1e3
        if df.plan is None:  # a command that looked like a query: already executed
            res = df.to_pandas()
        else:
            # lowering (+ a first-seen shape's compile, in the background: the first runs of a new
            # shape use the interpreter kernel) -- before a stream slot is held
            from ..engine.device_exec import async_compile

            tp = time.perf_counter()
            # (timeline: the caching allocator's free-everything-and-retry count around the statement
            # -- a retry frees every cached block of every stream, a device-wide stall)
            ar0 = _alloc_retries() if rec is not None else 0
            with async_compile():
                df.prepare()
            tl = time.perf_counter()
            with sess.engine.coalescer().scheduler.lease():
                tr = time.perf_counter()
                try:
                    res = df.run(token=token)  # the executor's columns, encoded without a DataFrame
                except torch.OutOfMemoryError:
                    # a temporary outside the slot arenas (a sort, a gather) found the HBM held by
                    # other slots' arenas and cached slot-0 tables: release those (not this slot's
                    # arena) and run the statement once more -- counted, so repeats show up
                    from ..engine.device_exec import release_device_memory, slot_arena
                    from ..engine.scheduler import current_slot
                    from ..utils.metrics import count_event

                    log.warning("statement ran out of device memory; releasing caches and retrying once")
                    count_event("statement_oom_retry")
                    release_device_memory(keep_arena=slot_arena(sess.engine.world.device(), current_slot()))
                    res = df.run(token=token)
                if rec is not None:
                    # the slot's stream is synchronised when the lease ends: run = host + GPU
                    rec.update(prepare_ms=(tl - tp) * 1e3, slot_wait_ms=(tr - tl) * 1e3,
                               run_ms=(time.perf_counter() - tr) * 1e3, alloc_retries=_alloc_retries() - ar0)
        return list(df.columns), [t for _, t in df.schema], res


def warm_up(session, statements) -> dict:
    """A server's warm-up before it takes clients (``hive_server --warmup FILE``): each statement is
    prepared (first-seen kernels compile) and run once on a leased execution slot, once more after
    the background compiles it started have finished (its final plan), and then every slot's device
    memory is sized for the largest of them (engine/device_exec.py presize_device_memory) -- the
    service then starts with its arenas, partition scratch and kernels in place."""
    from ..engine.device_exec import async_compile, presize_device_memory, wait_background_compiles

    sched = session.engine.coalescer().scheduler
    ran = 0
    for rnd in range(2):
        for st in statements:
            df = session.sql(st)
            if df.plan is None:
                continue
            with async_compile():
                df.prepare()
            with sched.lease():
                df.run()
            ran += 1
        if not wait_background_compiles():
            break
    out = presize_device_memory(session.engine.world.device(), sched.nslots)
    out["statements_run"] = ran
    return out


def _alloc_retries() -> int:
    return int(torch.cuda.memory_stats().get("num_alloc_retries", 0)) if torch.cuda.is_available() else 0


def make_server(session, host: str = "127.0.0.1", port: int = 10000, world=None, native: Optional[bool] = None):
    """The native-gateway server when its extension builds/loads (default), else the Python one."""
    if native is None:
        native = os.environ.get("SDO_NATIVE_GATEWAY", "1") != "0"
    if native:
        try:
            load_native()
            return NativeHiveServer(session, host, port, world=world)
        except Exception as e:  # noqa: BLE001
            log.warning("native gateway unavailable (%s); using the Python server", e)
    return HiveThriftServer(session, host, port, world=world)
