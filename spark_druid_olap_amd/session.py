"""Session: SQL entry point over the GPU engine (the reference's ``SPLSessionState`` + Spark
``SQLContext.sql`` + ``DruidStrategy``; ``asql/hive/sparklinedata/SPLSessionState.scala:77-190``).

    sess = Session()
    sess.register_datasource(ds)                    # a device-resident Druid index shard
    sess.register_table("orderLineItemPartSupplierBase", df_or_schema)
    sess.sql("CREATE TABLE t USING org.sparklinedata.druid OPTIONS (sourceDataframe ..., ...)")
    sess.sql("select l_returnflag, count(*) from t group by l_returnflag").collect()

Every rank of a multi-GPU job runs the same statements; ``DruidQuery`` leaves execute on the
rank's shard and merge over RCCL inside the engine, so results are global on every rank.
"""
from __future__ import annotations

import json
import threading
from collections import OrderedDict
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple, Iterator

import numpy as np
import pandas as pd

from .catalog.catalog import (CSV_PROVIDERS, DRUID_PROVIDERS, BaseTable, Catalog, DruidTable, ViewTable,
                              csv_loader)
from .catalog.history import DruidQueryHistory
from .catalog.options import Conf
from .catalog import views as V
from .query import spec as S
from .sql import ast as A
from .sql import plan as P
from .sql.analyzer import Analyzer
from .sql.druid_rewrite import DruidRewriter
from .sql.execute import Batch, Executor, FastStatement
from .sql.optimizer import optimize
from .sql.parser import ParseError, parse
from .sql.types import AnalysisError, series_to_list, to_series
from .utils import trace as T

_RUN_HELPERS: list = []


def _run_helpers():
    """(results_on_root, root_only_results, cancel scope), imported once (the engine imports lazily)."""
    if not _RUN_HELPERS:
        from .engine.executor import results_on_root, root_only_results
        from .utils.cancel import scope

        _RUN_HELPERS.append((results_on_root, root_only_results, scope))
    return _RUN_HELPERS[0]

_PANDAS_TO_SQL = {"i": "bigint", "u": "bigint", "f": "double", "b": "boolean", "M": "timestamp"}


def _infer_schema(df: pd.DataFrame) -> List[Tuple[str, str]]:
    out = []
    for c in df.columns:
        dt = df[c].dtype
        s = str(dt)
        if s == "Int64":
            out.append((c, "bigint"))
        elif s == "Float64":
            out.append((c, "double"))
        elif s == "boolean":
            out.append((c, "boolean"))
        else:
            out.append((c, _PANDAS_TO_SQL.get(dt.kind, "string")))
    return out


class DataFrame:
    """Result of ``Session.sql``: an optimized plan (lazy) or a command's rows."""

    def __init__(self, session: "Session", plan: Optional[P.Plan], names: List[str], sql: str = "",
                 batch: Optional[Batch] = None, analyzed: Optional[P.Plan] = None, rewrite_log=None):
        self.session = session
        self.plan = plan
        self.names = names
        self.sql_text = sql
        self._batch = batch
        self.analyzed = analyzed
        self.rewrite_log = rewrite_log or []
        self.last_stats: Dict[str, Any] = {}

    # -- execution ---------------------------------------------------------------------------
    def _run(self, token=None) -> Batch:
        if self._batch is not None:
            return self._batch
        if token is None:
            tmo = self.session.conf.typed("spark.sparklinedata.druid.query.timeout.ms")
            if tmo:
                from .utils.cancel import CancelToken

                token = CancelToken(tmo)
        results_on_root, root_only_results, scope = _run_helpers()
        t0 = time.perf_counter()
        if token is None:
            # projections over one pushed query (sql/execute.py FastStatement): no operator dispatch
            fast = self.__dict__.get("_fast")
            if fast is None:
                fast = self._fast = (FastStatement.compile(self.plan) or False) if self.plan is not None else False
            if fast:
                root_only = root_only_results() and self._root_only_safe()
                with results_on_root(root_only):
                    b, res, dst = self.session._with_sql(self.sql_text, lambda: fast.run(self.session))
                if b is not None:
                    self.last_stats = {"ms": (time.perf_counter() - t0) * 1e3, "druid": dst}
                    return b
                ex = Executor(self.session, token)
                ex.preload(fast.dq, res)  # the general operators finish from the same result
            else:
                ex = Executor(self.session, token)
        else:
            ex = Executor(self.session, token)
        # results on rank 0 only (the caller asked, engine/executor.py results_on_root) unless a
        # pushed query's spec is parameterized by another query's result: every rank needs those
        root_only = root_only_results() and self._root_only_safe()
        with scope(token), results_on_root(root_only):
            b = self.session._with_sql(self.sql_text, lambda: ex.run(self.plan))
        if isinstance(b, Batch):
            b.materialize_gathers()  # the statement's result rows are real arrays, not deferred gathers
        self.last_stats = {"ms": (time.perf_counter() - t0) * 1e3, "druid": ex.druid_stats}
        return b

    def prepared(self) -> "DataFrame":
        return self

    def prepare(self) -> "DataFrame":
        """Lower every pushed query whose spec is known up front (the GPU kernels of a first-seen
        shape compile here).  Servers call this before leasing an execution slot, so a compile
        never holds a stream slot; pushed queries parameterized by another query's result are
        prepared when they run.  One process only: several ranks prepare in broadcast order
        (server/spmd.py prepare_statement)."""
        if self.plan is not None and not self.session.engine.world.distributed:
            dqs = self.__dict__.get("_known_dqs")
            if dqs is None:  # (the plan is fixed: walk it once per cached statement)
                alld = P.find_all_deep(self.plan, P.DruidQuery)
                for dq in alld:
                    # the pushed queries of a subquery whose value parameterises another's filter
                    # sum exactly (sql/execute.py _subquery_param): prepared that way from the start
                    for d in S.find_deferred(dq.spec):
                        for sq in d.subqueries:
                            if isinstance(sq.query, P.Plan):
                                for x in P.find_all_deep(sq.query, P.DruidQuery):
                                    x.info["deterministic"] = True
                dqs = self._known_dqs = [dq for dq in alld if not S.find_deferred(dq.spec)]
            for dq in dqs:
                self.session.prepare_druid(dq)
        return self

    def _root_only_safe(self) -> bool:
        ok = self.__dict__.get("_root_ok")
        if ok is None:
            ok = self._root_ok = self.plan is not None and not any(
                S.find_deferred(dq.spec) for dq in P.find_all_deep(self.plan, P.DruidQuery))
        return ok

    def run(self, token=None) -> Batch:
        return self._run(token)

    def collect(self, token=None) -> List[tuple]:
        b = self._run(token)
        cols = [series_to_list(b.cols[r.rid], r.dtype) for r in b.refs]
        return list(zip(*cols)) if cols else [() for _ in range(b.n)]

    def to_pandas(self, token=None) -> pd.DataFrame:
        return self._run(token).to_pandas(self.names)

    toPandas = to_pandas

    def _stream_source(self, aggregates: bool = False):
        """(Limit n or None, DruidQuery) when the plan is Project/Filter operators over a pushed
        Select (the reference's push_project_and_filters path) -- or, with ``aggregates``, over a
        pushed groupBy: those can run page by page."""
        node, limit = self.plan, None
        if isinstance(node, P.Limit):
            limit, node = node.n, node.child
        while isinstance(node, (P.Project, P.Filter)):
            node = node.child
        kinds = (S.SelectSpec, S.GroupByQuerySpec) if aggregates else (S.SelectSpec,)
        if isinstance(node, P.DruidQuery) and isinstance(node.spec, kinds) and \
                not S.find_deferred(node.spec) and not node.info.get("historical"):
            return limit, node
        return None, None

    def agg_streamable(self) -> bool:
        """Project/Filter over a pushed groupBy that can be answered page by page: no HAVING,
        limitSpec or theta sketch, and a key space (the product of its plain dimensions' dictionary
        sizes) of at least ``engine/executor.py STREAM_MIN_GROUPS``.  Decided from the plan and the
        catalog alone -- no lowering, no collective -- so the multi-rank dispatcher can ask it on
        rank 0 while routing a statement (server/spmd.py _assign)."""
        if self.plan is None:
            return False
        _, dq = self._stream_source(aggregates=True)
        spec = getattr(dq, "spec", None)
        if not isinstance(spec, S.GroupByQuerySpec) or spec.having is not None or spec.limitSpec is not None:
            return False
        if any(isinstance(a, S.ThetaSketchAggregationSpec) for a in (spec.aggregations or [])):
            return False
        from .engine import executor as E

        ds = dq.relation.info.datasource
        space = 1
        for d in spec.dimensions or []:
            col = ds.dims.get(getattr(d, "dimension", None)) if type(d) is S.DefaultDimensionSpec else None
            if col is None:
                return False
            space *= max(1, col.cardinality)
        return space >= E.STREAM_MIN_GROUPS

    def _run_pages(self, dq, limit, pages, token):
        left = limit
        for res in pages:
            ex = Executor(self.session, token)
            ex.preload(dq, res)
            b = self.session._with_sql(self.sql_text, lambda: ex.run(self.plan if limit is None else self.plan.child))
            out = b.to_pandas(self.names)
            if left is not None:
                out = out.iloc[:left]
                left -= len(out)
            if len(out):
                yield out
            if left is not None and left <= 0:
                return

    def iter_batches(self, page_rows: Optional[int] = None, token=None) -> Iterator[pd.DataFrame]:
        """The result as a stream of pandas pages: a Select-backed plan is executed one Druid page
        at a time (``spark.sparklinedata.druid.selectquery.pagesize`` rows per shard page, the
        reference's DruidSelectResultIterator.scala:116-137 cursor), so host memory holds one page;
        any other plan is computed, then sliced."""
        page_rows = int(page_rows or self.session.conf.typed("spark.sparklinedata.druid.selectquery.pagesize"))
        limit, dq = (None, None) if self.plan is None else self._stream_source()
        if dq is None and self.agg_streamable():
            # a large pushed groupBy: each page's groups are decoded and copied from the device as
            # they are pulled (engine/executor.py iter_pages)
            limit, dq = self._stream_source(aggregates=True)
            prep = self.session.prepare_druid(dq)
            if getattr(prep, "streamable", lambda: False)():
                # several ranks: only rank 0 pages through the groups (the multi-rank server answers
                # from rank 0; the peers' cursors end after the first, collective, step)
                root_only = self.session.engine.world.distributed and self._root_only_safe()
                yield from self._run_pages(dq, limit, prep.iter_pages(page_rows, root_only), token)
                return
            dq = None
        if dq is None:
            df = self.to_pandas(token)
            for a in range(0, max(len(df), 1), page_rows):
                if a < len(df) or a == 0:
                    yield df.iloc[a: a + page_rows].reset_index(drop=True)
            return
        yield from self._run_pages(dq, limit, self.session.iter_select_pages(dq, page_rows), token)

    def toLocalIterator(self, page_rows: Optional[int] = None) -> Iterator[tuple]:
        """Rows one at a time over ``iter_batches`` (Spark's ``DataFrame.toLocalIterator``)."""
        for page in self.iter_batches(page_rows):
            yield from page.itertuples(index=False, name=None)

    def count(self) -> int:
        return self._run().n

    @property
    def columns(self) -> List[str]:
        return list(self.names)

    @property
    def schema(self) -> List[Tuple[str, str]]:
        refs = self.plan.output if self.plan is not None else self._batch.refs
        return [(n, r.dtype) for n, r in zip(self.names, refs)]

    # -- introspection (plan-shape tests, DruidPlanner.getDruidQuerySpecs) ----------------------
    def druid_queries(self) -> List[P.DruidQuery]:
        return P.find_all_deep(self.plan, P.DruidQuery) if self.plan is not None else []

    def druid_query_specs(self) -> List[S.QuerySpec]:
        return [d.spec for d in self.druid_queries()]

    def explain(self, extended: bool = False) -> str:
        if self.plan is None:
            return "<command>"
        s = ""
        if extended and self.analyzed is not None:
            s += "== Analyzed Logical Plan ==\n" + self.analyzed.tree_string() + "\n"
        s += "== Physical Plan ==\n" + self.plan.tree_string()
        return s

    def show(self, n: int = 20) -> None:
        print(self.to_pandas().head(n).to_string())

    def __repr__(self):
        return f"DataFrame[{', '.join(f'{n}: {t}' for n, t in self.schema)}]"


class Session:
    def __init__(self, engine=None, conf: Optional[Dict[str, Any]] = None, world=None):
        if engine is None:
            from .engine.executor import Engine

            engine = Engine(world)
        self.engine = engine
        self.conf = Conf(conf)
        self.catalog = Catalog()
        self.history = DruidQueryHistory(int(self.conf.typed("sparkline.queryhistory.maxsize")))
        from .utils.metrics import ServerMetrics

        self.metrics = ServerMetrics()  # per-endpoint latency percentiles / QPS (servers record)
        self._plan_cache: "OrderedDict[tuple, DataFrame]" = OrderedDict()
        self._lock = threading.RLock()
        self._tl = threading.local()
        from .modules import load_modules

        self.modules = load_modules(self)
        self.discovery = None
        if self.conf.get("spark.sparklinedata.druid.discovery", "true") not in ("false", False):
            self.attach_discovery(self.conf.get("spark.sparklinedata.druid.zkHost", "localhost"))

    def new_session(self) -> "Session":
        """A client session over the same engine, tables and datasources with its own ``SET``
        configuration, current database, temporary views and plan cache (Spark's
        ``SparkSession.newSession``; one per HiveServer2 client session)."""
        s = Session.__new__(Session)
        s.engine = self.engine
        s.conf = self.conf.copy()
        s.catalog = self.catalog.session_view()
        s.history = self.history
        s.metrics = self.metrics
        # plans (and their prepared GPU queries and per-slot device buffers) are shared by every
        # session whose statement text, conf, current database and temp views match (the cache key)
        s._plan_cache = self._plan_cache
        s._lock = self._lock
        s._tl = threading.local()
        s.modules = self.modules
        s.discovery = self.discovery
        s.parent = self
        return s

    def attach_discovery(self, druid_host: str = "localhost", druid_path: str = "/druid",
                         qualify_names: bool = False):
        """Join the service registry named by a ``druidHost`` connect string (client/discovery.py)."""
        from .client.discovery import Discovery, registry_for

        self.discovery = Discovery(registry_for(druid_host), druid_path, qualify_names)
        self.catalog.cluster.attach_discovery(self.discovery, self.engine.world.rank)
        return self.discovery

    # ------------------------------------------------------------------------------ extension points
    def register_udf(self, name: str, fn, return_type: str = "string", vectorized: bool = False) -> None:
        """Register a scalar SQL function.  ``fn`` takes Python values (NULL-propagating, called per
        row) or, with ``vectorized=True``, pandas Series/scalars and returns the same shape.  Over a
        Druid dimension the function is still pushed down: it is evaluated once per dictionary
        entry, like every other single-dimension expression."""
        from .sql import functions as F

        if vectorized:
            impl = lambda args, ts, n: fn(*args)  # noqa: E731
        else:
            impl = F._map_scalar(fn, return_type)
        F._FUNCS[name.lower()] = F.Fn(name.lower(), lambda ts, t=return_type: t, impl)
        self._plan_cache.clear()

    # ------------------------------------------------------------------------------ registration
    def register_datasource(self, ds, name: Optional[str] = None) -> None:
        """Make a device-resident datasource shard queryable (the 'Druid cluster' contents)."""
        self._global_interval(ds)
        self.catalog.cluster.register(ds, name)
        self._plan_cache.clear()

    def _global_interval(self, ds) -> None:
        from .sql.druid_rewrite import data_interval

        if getattr(ds, "global_interval_ms", None) is not None:
            return
        lo, hi = data_interval(ds)
        w = self.engine.world
        if w.size > 1:
            lo = -w.max_float(-float(lo))
            hi = w.max_float(float(hi))
        ds.global_interval_ms = (int(lo), int(hi))

    def register_table(self, name: str, df: Optional[pd.DataFrame] = None,
                       schema: Optional[Sequence[Tuple[str, str]]] = None, loader=None,
                       temporary: bool = False) -> BaseTable:
        db, tname = self.catalog._split(name)
        db = db or self.catalog.current_db
        if schema is None:
            if df is None:
                raise AnalysisError("register_table needs data or a schema")
            schema = _infer_schema(df)
        schema = [(c, _norm_type(t)) for c, t in schema]
        t = BaseTable(db, tname, list(schema), data=None, loader=(lambda d=df: d) if df is not None else loader)
        self.catalog.register(t, temporary=temporary)
        self._plan_cache.clear()
        return t

    def table(self, name: str) -> DataFrame:
        return self.sql(f"select * from {name}")

    # ------------------------------------------------------------------------------ SQL
    def sql(self, text: str) -> DataFrame:
        for m in self.modules:
            p = getattr(m, "parse", None)
            if p is not None:
                r = p(text, self)
                if r is not None:
                    return r
        from .utils import trace as T

        # a statement planned before (same text, catalog, database, temp views, SET values) skips
        # the parser too: the cache only holds queries
        hit = self._cached_plan(text)
        if hit is not None:
            return hit
        try:
            with T.span("sdo.parse"):
                st = parse(text)
        except ParseError as pe:
            raise ParseError(f"{pe}\n\n== SQL ==\n{text}") from None
        if isinstance(st, (A.Select, A.SetOp, A.With)):
            with T.span("sdo.plan"):
                return self._query(text, st)
        return self._command(text, st)

    PLAN_CACHE_MAX = 4096

    def _plan_key(self, text: str):
        # statements over the d$* metadata views are planned afresh (their rows are the metadata
        # at planning time); everything else is cached by text + catalog / registry / conf state
        if "d$" in text.lower() or not self.conf.typed("spark.sparklinedata.druid.planCache.enabled"):
            return None
        return (text, self.catalog.version, self.catalog.current_db, id(self.catalog.temp) if self.catalog.temp else 0,
                self.catalog.cluster.generation, self.conf.cache_key())

    def _cached_plan(self, text: str) -> Optional[DataFrame]:
        key = self._plan_key(text)
        if key is None:
            return None
        hit = self._plan_cache.get(key)
        if hit is not None:
            try:
                self._plan_cache.move_to_end(key)  # LRU (a dashboard's few thousand parameterizations)
            except KeyError:
                pass
        return hit

    def _query(self, text: str, st) -> DataFrame:
        key = self._plan_key(text)
        if key is not None:
            hit = self._plan_cache.get(key)
            if hit is not None:
                return hit
        df = self.plan(text, st)
        if key is not None:
            with self._lock:
                self._plan_cache[key] = df
                while len(self._plan_cache) > self.PLAN_CACHE_MAX:
                    self._plan_cache.popitem(last=False)
        return df

    def plan(self, text: str, st=None) -> DataFrame:
        st = st if st is not None else parse(text)
        an = Analyzer(self.catalog, self)
        analyzed = an.analyze(st)
        names = [r.name for r in analyzed.output]
        rw = DruidRewriter(self)
        phys = self._physical(analyzed, rw)
        if self.conf.typed("spark.sparklinedata.druid.debug.transformations"):
            import logging

            logging.getLogger("sdo.planner").info("rewrite log:\n%s\nplan:\n%s", "\n".join(rw.log),
                                                  phys.tree_string())
        return DataFrame(self, phys, names, text, analyzed=analyzed, rewrite_log=rw.log)

    def _physical(self, analyzed: P.Plan, rw: "DruidRewriter") -> P.Plan:
        """optimize -> module logical rules -> Druid rewrite -> module physical rules.  Subquery
        plans inside expressions (scalar / IN / EXISTS) go through the same pipeline first, so a
        scalar subquery over a Druid table is itself a pushed GPU query (Spark plans them as
        separate physical plans too, ``ScalarSubquery`` / ``PlanSubqueries``)."""
        for sq in P.subquery_exprs(analyzed):
            if not getattr(sq, "_planned", False):
                object.__setattr__(sq, "query", self._physical(sq.query, rw))
                object.__setattr__(sq, "_planned", True)
        opt = optimize(analyzed, self.conf)
        for m in self.modules:
            for rule in getattr(m, "logical_rules", []) or []:
                opt = rule(opt, self) or opt
        phys = rw.rewrite(opt)
        if self.conf.typed("spark.sparklinedata.druid.window.rankone.pushdown"):
            from .sql.window import push_rank_one

            phys = push_rank_one(phys)  # rank() = 1 over a pushed aggregate: a device pre-filter
        for m in self.modules:
            for rule in getattr(m, "physical_rules", []) or []:
                phys = rule(phys, self) or phys
        return phys

    def _with_sql(self, sql: str, fn):
        prev = getattr(self._tl, "sql", None)
        self._tl.sql = sql
        try:
            return fn()
        finally:
            self._tl.sql = prev

    # ------------------------------------------------------------------------------ druid exec
    def iter_select_pages(self, dq: P.DruidQuery, page_rows: int) -> Iterator[Any]:
        """Pages of a pushed Select: the engine computes the shard's selected rows once and each
        page gathers ``page_rows`` rows per shard (engine/executor.py run_page); the paging
        identifiers of one page are the cursor of the next."""
        spec = dq.spec
        prep = self.engine.prepare(spec.copy(pagingSpec=S.PagingSpec({}, page_rows)), dq.relation.info.datasource)
        ident: Dict[str, int] = {}
        while True:
            res = prep.run_page(S.PagingSpec(dict(ident), page_rows))
            if res.num_rows == 0:
                return
            yield res
            ident = res.paging

    def run_druid_sets(self, dqs: List[P.DruidQuery]):
        """Grouping-set branches from one engine scan (engine/executor.py execute_grouping_sets);
        None when they cannot be fused (each branch then runs on its own)."""
        if not self.conf.typed("spark.sparklinedata.druid.fuse.groupingsets"):
            return None
        ds = dqs[0].relation.info.datasource
        t0 = time.perf_counter()
        out_types = [{n: t for n, t, k in dq.columns if k == "value"} for dq in dqs]
        res = self.engine.execute_sets([dq.spec for dq in dqs], ds, out_types)
        if res is not None and self.conf.typed("spark.sparklinedata.enable.druid.query.history"):
            ms = (time.perf_counter() - t0) * 1e3
            for dq, r in zip(dqs, res):
                self.history.record(dq.spec, r.stats.get("exec_ms", ms), ms, r.num_rows,
                                    f"gpu:0-{self.engine.world.size - 1}", getattr(self._tl, "sql", None),
                                    len(ds.segments))
        return res

    def run_druid(self, dq: P.DruidQuery):
        ds = dq.relation.info.datasource
        spec = dq.spec
        t0 = time.perf_counter()
        prep = self.prepare_druid(dq)
        with T.span(f"sdo.druid.{spec.queryType}"):
            res = prep.run()
        if isinstance(spec, S.TimeSeriesQuerySpec) and res.num_rows == 0:
            res = _empty_global_agg(res, spec)
        ms = (time.perf_counter() - t0) * 1e3
        if self.conf.typed("spark.sparklinedata.enable.druid.query.history"):
            self.history.record(spec, res.stats.get("exec_ms", ms), ms, res.num_rows,
                                f"gpu:0-{self.engine.world.size - 1}", getattr(self._tl, "sql", None),
                                len(ds.segments))
        return res

    def prepare_druid(self, dq: P.DruidQuery):
        """The engine's prepared query for pushed query ``dq`` (lowered once, cached on the plan
        node).  Lowering may issue collectives (cluster-wide FD tables, row estimates), so the SPMD
        server calls this in broadcast order on every rank before a statement runs on a slot."""
        ds = dq.relation.info.datasource
        spec = dq.spec
        run_spec = spec
        if isinstance(spec, S.SelectSpec):
            # one page holding every row (the reference's paging loop, DruidSelectResultIterator.scala:116-137,
            # collapsed: the scan compacts on device and ships all selected rows at once)
            run_spec = spec.copy(pagingSpec=S.PagingSpec({}, 2 ** 31 - 1))
        det = bool(self.conf.typed("spark.sparklinedata.druid.deterministic")) or bool(dq.info.get("deterministic"))
        if det:
            ctx = getattr(run_spec, "context", None)
            run_spec = run_spec.copy(context=ctx.copy(deterministic=True) if ctx is not None
                                     else S.QuerySpecContext(deterministic=True))
        prep = getattr(dq, "_prepared", None)
        # (an interim plan -- first-seen kernels compiling in the background, engine/device_exec.py
        # async_compile -- is replaced once they are all compiled)
        stale = lambda p: p is None or getattr(dq, "_prepared_spec", None) is not spec or \
            getattr(p, "deterministic", False) != (det or getattr(p, "deterministic", False)) or \
            (bool(getattr(p, "jit_pending", None)) and all(f.done() for f in p.jit_pending))  # noqa: E731
        if stale(prep):
            # concurrent sessions share cached plans: prepare once -- under a lock of this pushed
            # query only, so preparing (and compiling) one statement never blocks another's
            lock = dq.__dict__.get("_prep_lock")
            if lock is None:
                with self._lock:
                    lock = dq.__dict__.setdefault("_prep_lock", threading.Lock())
            with lock:
                prep = getattr(dq, "_prepared", None)
                if stale(prep):
                    from .engine.device_exec import prepare_collecting

                    with T.span("sdo.lower"):
                        prep, pending = prepare_collecting(
                            lambda: self.engine.prepare(run_spec, ds, dq.info.get("historical")))
                    from .utils.metrics import count_event

                    old = getattr(dq, "_prepared", None)
                    count_event("plan_prepare" if old is None else "plan_reprepare_jit" if getattr(old, "jit_pending", None)
                                else "plan_reprepare_spec" if getattr(dq, "_prepared_spec", None) is not spec
                                else "plan_reprepare", detail=f"{type(spec).__name__} det={det} "
                                f"old_det={getattr(old, 'deterministic', None)} {str(getattr(spec, 'filter', ''))[:120]}")
                    if pending:
                        prep.jit_pending = pending
                    # output SQL types: large results decode numeric dictionary keys on the device
                    # (and integer outputs of string-valued extractions: 'yyyy' time formats)
                    prep.out_types = {n: t for n, t, k in dq.columns
                                      if k == "value" or (k == "string" and t in ("tinyint", "smallint", "int", "bigint"))}
                    # rank() = 1 window above (sql/window.py push_rank_one): device pre-filter
                    prep.partition_extreme = dq.info.get("partition_extreme")
                    # device work the prepare launched on this thread's stream (descriptor-side
                    # tables, LUTs, packed copies) completes before other slots -- whose streams
                    # were ordered after the default stream when they were leased, possibly before
                    # this -- can pick the plan up (utils/streams.py)
                    from .utils.streams import publish

                    publish(prep, ds.device if hasattr(ds, "device") else None)
                    dq._prepared = prep
                    dq._prepared_spec = spec
        return prep

    # ------------------------------------------------------------------------------ commands
    def _rows_df(self, cols: List[Tuple[str, str]], rows: List[tuple]) -> DataFrame:
        refs = [A.Ref(A.new_id(), c, t) for c, t in cols]
        data = {}
        for i, r in enumerate(refs):
            data[r.rid] = to_series(pd.Series([row[i] for row in rows], dtype=object), r.dtype)
        return DataFrame(self, None, [c for c, _ in cols], batch=Batch(refs, data, len(rows)))

    def _command(self, text: str, st) -> DataFrame:
        cat = self.catalog
        if isinstance(st, A.CreateTable):
            return self._create_table(st)
        if isinstance(st, A.CreateView):
            db, name = cat._split(st.name)
            v = ViewTable(db or cat.current_db, name, st.query, st.text)
            if not st.replace and cat.lookup(st.name) is not None and not st.temporary:
                raise AnalysisError(f"View {name} already exists")
            cat.register(v, temporary=st.temporary)
            self._plan_cache.clear()
            return self._rows_df([], [])
        if isinstance(st, A.DropTable):
            cat.drop(st.name, st.if_exists)
            self._plan_cache.clear()
            return self._rows_df([], [])
        if isinstance(st, A.CreateDatabase):
            cat.create_database(st.name, st.if_not_exists)
            return self._rows_df([], [])
        if isinstance(st, A.UseDatabase):
            cat.use(st.name)
            self._plan_cache.clear()
            return self._rows_df([], [])
        if isinstance(st, A.SetConf):
            if st.key is None:
                items = sorted(self.conf.items().items())
                return self._rows_df([("key", "string"), ("value", "string")], items)
            if st.value is None:
                return self._rows_df([("key", "string"), ("value", "string")],
                                     [(st.key, self.conf.get(st.key, "<undefined>"))])
            self.conf.set(st.key, st.value)
            self._plan_cache.clear()
            return self._rows_df([("key", "string"), ("value", "string")], [(st.key, st.value)])
        if isinstance(st, A.ShowTables):
            rows = [(t.db, t.name.lower(), t in cat.temp.values()) for t in cat.tables(st.db)]
            return self._rows_df([("database", "string"), ("tableName", "string"), ("isTemporary", "boolean")], rows)
        if isinstance(st, A.Describe):
            t = self.lookup_table(st.name)
            return self._rows_df([("col_name", "string"), ("data_type", "string"), ("comment", "string")],
                                 [(c, ty, None) for c, ty in t.schema])
        if isinstance(st, A.CacheTable):
            t = cat.get(st.name)
            if isinstance(t, BaseTable):
                t.cached = not st.uncache
                if t.cached:
                    t.frame()
            return self._rows_df([], [])
        if isinstance(st, A.ClearDruidCache):
            cat.cluster.clear_cache(st.host)
            self._plan_cache.clear()
            return self._rows_df([], [])
        if isinstance(st, A.ExecuteDruidQuery):
            return self._execute_query(st)
        if isinstance(st, A.ExplainDruidRewrite):
            return self._explain_rewrite(st)
        if isinstance(st, A.Explain):
            df = self.plan("", st.query)
            return self._rows_df([("plan", "string")], [(df.explain(st.extended),)])
        raise AnalysisError(f"unsupported statement {type(st).__name__}")

    def lookup_table(self, name):
        if isinstance(name, tuple) and len(name) == 1 and name[0].lower() in V.VIEWS:
            return self.metadata_view(name[0])
        return self.catalog.get(name)

    def metadata_view(self, name: str) -> BaseTable:
        df = V.VIEWS[name.lower()](self)
        return BaseTable("default", name.lower(), V.schema_of(df), data=df)

    def _create_table(self, st: A.CreateTable) -> DataFrame:
        cat = self.catalog
        if cat.lookup(st.name) is not None:
            if st.if_not_exists:
                return self._rows_df([], [])
            raise AnalysisError(f"Table {'.'.join(st.name)} already exists")
        prov = (st.provider or "").lower()
        db, name = cat._split(st.name)
        db = db or cat.current_db
        if prov in DRUID_PROVIDERS:
            t = cat.create_druid_relation(st.name, st.options)
            cat.register(t, temporary=st.temporary)
        elif st.as_query is not None:
            df = self.sql_ast(st.as_query)
            data = df.to_pandas()
            schema = list(df.schema)
            cat.register(BaseTable(db, name, schema, data=None, loader=lambda d=data: d), temporary=st.temporary)
        elif prov in CSV_PROVIDERS:
            path = st.options.get("path")
            if path is None:
                raise AnalysisError("csv tables need a path option")
            schema = [(c.name, c.dtype) for c in st.columns]
            cat.register(BaseTable(db, name, schema, loader=csv_loader(path, schema, st.options), provider=prov,
                                   options=st.options), temporary=st.temporary)
        elif prov in ("parquet", "json", "orc"):
            path = st.options.get("path")
            schema = [(c.name, c.dtype) for c in st.columns] or None

            def load(path=path, prov=prov):
                if prov == "parquet":
                    return pd.read_parquet(path)
                if prov == "json":
                    return pd.read_json(path, lines=True)
                raise AnalysisError("orc is not supported")
            if schema is None:
                probe = load()
                schema = _infer_schema(probe)
            cat.register(BaseTable(db, name, schema, loader=load, provider=prov, options=st.options),
                         temporary=st.temporary)
        elif not prov:
            schema = [(c.name, c.dtype) for c in st.columns]
            empty = pd.DataFrame({c: to_series([], t) for c, t in schema})
            cat.register(BaseTable(db, name, schema, data=None, loader=lambda d=empty: d), temporary=st.temporary)
        else:
            raise AnalysisError(f"Failed to find data source: {st.provider}")
        self._plan_cache.clear()
        return self._rows_df([], [])

    def sql_ast(self, st) -> DataFrame:
        return self.plan("", st)

    def _execute_query(self, st: A.ExecuteDruidQuery) -> DataFrame:
        """``ON DRUIDDATASOURCE t EXECUTE QUERY <json>`` (PlanUtil.logicalPlan, asql/util/PlanUtil.scala:48-61)."""
        from .query.spec import query_from_json

        t = self.catalog.get(st.table)
        if not isinstance(t, DruidTable):
            raise AnalysisError(f"{'.'.join(st.table)} is not a Druid relation")
        spec = query_from_json(json.loads(st.json_text))
        nseg = None
        if st.historical:  # USING HISTORICAL: segment-batched partials merged by the engine
            nseg = max(1, min(t.info.options.num_segments_per_query(self.conf), 1 << 30))
        res = self.engine.execute(spec, t.info.datasource, nseg)
        if self.conf.typed("spark.sparklinedata.enable.druid.query.history"):
            self.history.record(spec, res.stats.get("exec_ms", 0.0), res.stats.get("exec_ms", 0.0), res.num_rows,
                                f"gpu:0-{self.engine.world.size - 1}", None)
        from .engine.columns import materialize

        cols = []
        rows_cols = []
        for c in res.columns:
            arr = materialize(res.data[c])
            k = np.asarray(arr).dtype.kind
            t_ = "bigint" if k in "iu" else "double" if k == "f" else "string"
            cols.append((c, t_))
            rows_cols.append([x.item() if isinstance(x, np.generic) else x for x in np.asarray(arr).tolist()])
        rows = list(zip(*rows_cols)) if rows_cols else []
        return self._rows_df(cols, rows)

    def _explain_rewrite(self, st: A.ExplainDruidRewrite) -> DataFrame:
        """``EXPLAIN DRUID REWRITE`` (ExplainDruidRewrite.run, DruidMetadataCommands.scala:58-77)."""
        from .planner.cost import explain_cost

        df = self.plan("", st.query)
        lines = df.plan.tree_string().rstrip("\n").split("\n")
        for i, dq in enumerate(df.druid_queries()):
            lines.append(f"DruidQuery({i}) details ::")
            lines.append(json.dumps(dq.spec.to_json(), indent=2))
            lines.extend(explain_cost(self, dq).split("\n"))
        return self._rows_df([("plan", "string")], [(l,) for l in lines])


def _norm_type(t: str) -> str:
    from .sql.parser import TYPE_NAMES

    t = t.strip()
    u = t.upper()
    if "(" in u:
        head = u[: u.index("(")]
        if TYPE_NAMES.get(head) == "decimal":
            return "decimal" + t[t.index("("):].replace(" ", "")
        return TYPE_NAMES.get(head, t.lower())
    return TYPE_NAMES.get(u, t.lower())


def _empty_global_agg(res, spec):
    """SQL global aggregates return one row even over no input (count = 0, others NULL)."""
    from .engine.executor import QueryResult

    data = {}
    cols = list(res.columns) if res.columns else ["timestamp"] + [a.name for a in spec.aggregations]
    for c in cols:
        data[c] = np.array([0 if c in _count_names(spec) else np.nan], dtype=object)
    return QueryResult(cols, data, res.query_type, res.stats)


def _count_names(spec) -> set:
    out = set()
    for a in spec.aggregations or []:
        if isinstance(a, S.FunctionAggregationSpec) and a.type == "count":
            out.add(a.name)
        if isinstance(a, S.FilteredAggregationSpec):
            out.add(a.name)
        if isinstance(a, S.CardinalityAggregationSpec):
            out.add(a.name)
    return out
