"""Select cursor + streamed results (K16 / C4 / L2 result iterators).

The reference pages Select queries (``asd/DruidSelectResultIterator.scala:116-137``, 10,000 rows
per page, ``asd/DruidPlanner.scala:78-81``) and streams query results into Spark
(``asd/DruidQueryResultIterator.scala:58-90``).  Here: a prepared Select computes the shard's rows
once, every page is a device gather, ``DataFrame.iter_batches`` executes Project/Filter plans one
page at a time, and the Thrift server streams those pages to the client."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from spark_druid_olap_amd.engine.columns import materialize
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.session import Session

SEL = S.SelectSpec("tpch", ["s_nation", "l_shipmode"], ["l_extendedprice", "l_quantity"],
                   filter=S.SelectorFilterSpec("s_region", "ASIA"), intervals=["1992-01-01/1999-01-01"])


def _rows(res):
    return list(zip(materialize(res.data["timestamp"]).tolist(), materialize(res.data["s_nation"]).tolist(),
                    materialize(res.data["l_shipmode"]).tolist(), res.data["l_extendedprice"].tolist(),
                    res.data["l_quantity"].tolist()))


def _all_pages(pq, thr, world=1):
    out, ident, pages = [], {}, 0
    while True:
        r = pq.run_page(S.PagingSpec(dict(ident), thr))
        if r.num_rows == 0:
            return out, pages
        assert r.num_rows <= thr * world  # threshold rows per shard and page
        out += _rows(r)
        ident = r.paging
        pages += 1


@pytest.mark.parametrize("descending", [False, True])
def test_pages_cover_the_full_select_once(ds_small, descending):
    eng = Engine(use_native=False)
    q = SEL.copy(descending=descending)
    full = eng.execute(q.copy(pagingSpec=S.PagingSpec({}, 10 ** 9)), ds_small)
    pq = eng.prepare(q, ds_small)
    got, pages = _all_pages(pq, 997)
    assert got == _rows(full)
    assert pages == -(-full.num_rows // 997)
    # the selected rows are computed once per prepared query, not per page
    assert getattr(pq, "_sel_rows", None) is not None


def _session(ds, df):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False,
                         extra_options=', nonAggregateQueryHandling "push_project_and_filters"'))
    return s


SQL = ("select s_nation, l_extendedprice * 2 as x, l_quantity from orderLineItemPartSupplier "
       "where s_region = 'ASIA' and l_quantity > 10")


def test_dataframe_iter_batches_streams_select(ds_small, df_small):
    s = _session(ds_small, df_small)
    d = s.sql(SQL)
    assert isinstance(d.druid_query_specs()[0], S.SelectSpec)
    assert d._stream_source()[1] is not None
    pages = list(d.iter_batches(page_rows=500))
    assert len(pages) > 3 and all(len(p) <= 500 for p in pages)
    streamed = [tuple(r) for p in pages for r in p.itertuples(index=False, name=None)]
    assert sorted(streamed) == sorted(d.collect())
    assert list(d.toLocalIterator(page_rows=333)) == streamed or \
        sorted(d.toLocalIterator(page_rows=333)) == sorted(streamed)
    # a limit on top stops the cursor early
    lim = s.sql(SQL + " limit 700")
    got = [r for p in lim.iter_batches(page_rows=250) for r in p.itertuples(index=False, name=None)]
    assert len(got) == 700


def test_non_streamable_plans_fall_back_to_slices(ds_small, df_small):
    s = _session(ds_small, df_small)
    d = s.sql("select s_nation, count(*) from orderLineItemPartSupplier group by s_nation")
    assert d._stream_source()[1] is None
    pages = list(d.iter_batches(page_rows=10))
    assert sum(len(p) for p in pages) == 25


def test_thrift_server_streams_pages(ds_small, df_small):
    from spark_druid_olap_amd.server.hive_client import connect
    from spark_druid_olap_amd.server.hive_server import HiveThriftServer

    s = _session(ds_small, df_small)
    s.conf.set("spark.sparklinedata.druid.selectquery.pagesize", "300")
    srv = HiveThriftServer(s, port=0).start()
    try:
        with connect(port=srv.port) as c:
            cur = c.cursor()
            cur.arraysize = 128
            rows = cur.execute(SQL).fetchall()
        assert sorted(rows) == sorted(s.sql(SQL).collect())
        op = next(iter(srv.ops.values()), None)
        if op is not None:  # streamed: only the unread tail stays buffered
            assert op.factory is not None and len(op.cols[0]) <= 300 + 128 + 1
    finally:
        srv.stop()


GB_SQL = ("select o_orderkey, l_linenumber, count(*) as c, sum(l_extendedprice) as s "
          "from orderLineItemPartSupplier where l_quantity > 10 group by o_orderkey, l_linenumber")


def test_large_groupby_streams_pages(ds_small, df_small, monkeypatch):
    """A groupBy over a large key space streams: the merged groups stay in device / engine memory
    and each page is finalized when pulled (engine/executor.py iter_pages)."""
    from spark_druid_olap_amd.engine import executor as E

    monkeypatch.setattr(E, "STREAM_MIN_GROUPS", 1000)
    s = _session(ds_small, df_small)
    d = s.sql(GB_SQL)
    assert isinstance(d.druid_query_specs()[0], S.GroupByQuerySpec)
    assert d._stream_source()[1] is None and d.agg_streamable()
    calls = []
    real = E.PreparedQuery.iter_pages

    def spy(self, page_rows, root_only=None):
        calls.append(page_rows)
        yield from real(self, page_rows, root_only)

    monkeypatch.setattr(E.PreparedQuery, "iter_pages", spy)
    pages = list(d.iter_batches(page_rows=700))
    assert calls == [700] and len(pages) > 3 and all(len(p) <= 700 for p in pages)
    streamed = sorted(tuple(r) for p in pages for r in p.itertuples(index=False, name=None))
    assert streamed == sorted(d.collect())
    exp = df_small[df_small.l_quantity > 10].groupby(["o_orderkey", "l_linenumber"]).size()
    assert len(streamed) == len(exp)
    lim = s.sql(GB_SQL + " limit 900")  # a limit above the pushed groupBy stops the pages early
    assert sum(len(p) for p in lim.iter_batches(page_rows=400)) == 900
    # small key spaces and host-ordered results are not streamed
    assert not s.sql("select s_nation, count(*) from orderLineItemPartSupplier group by s_nation").agg_streamable()
    assert not s.sql(GB_SQL.replace("group by", "and 1 = 1 group by") + " having count(*) > 1").agg_streamable()


def test_thrift_server_streams_groupby_pages(ds_small, df_small, monkeypatch):
    from spark_druid_olap_amd.engine import executor as E
    from spark_druid_olap_amd.server.hive_client import connect
    from spark_druid_olap_amd.server.hive_server import HiveThriftServer

    monkeypatch.setattr(E, "STREAM_MIN_GROUPS", 1000)
    s = _session(ds_small, df_small)
    s.conf.set("spark.sparklinedata.druid.selectquery.pagesize", "500")
    srv = HiveThriftServer(s, port=0).start()
    try:
        with connect(port=srv.port) as c:
            cur = c.cursor()
            cur.arraysize = 200
            rows = cur.execute(GB_SQL).fetchall()
            op = next(iter(srv.ops.values()), None)
            assert op is not None and op.factory is not None
        assert sorted(rows) == sorted(s.sql(GB_SQL).collect())
    finally:
        srv.stop()


def _free_port():
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    p = s_.getsockname()[1]
    s_.close()
    return p


def _rank_pages(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    import pickle

    from spark_druid_olap_amd.parallel.world import init_world

    w = init_world(backend="gloo")
    ds = tpch.to_datasource(tpch.generate_flat(0.004, "cpu", rank=rank, world=world), profile="bench")
    eng = Engine(w, use_native=False)
    pq = eng.prepare(SEL, ds)
    got, pages = _all_pages(pq, 211, world)
    full = eng.execute(SEL.copy(pagingSpec=S.PagingSpec({}, 10 ** 9)), ds)
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump({"got": got, "full": _rows(full), "pages": pages}, f)
    w.barrier()


def test_two_rank_cursor_gathers_every_shard():
    import pickle

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_pages, args=(2, _free_port(), d), nprocs=2, join=True)
        r = [pickle.load(open(os.path.join(d, f"r{i}.pkl"), "rb")) for i in range(2)]
    # every rank sees the same merged pages, and they cover both shards exactly once
    assert r[0]["got"] == r[1]["got"]
    assert sorted(r[0]["got"]) == sorted(r[0]["full"])
    assert len(r[0]["got"]) == len(set(r[0]["got"])) or len(r[0]["got"]) == len(r[0]["full"])


@pytest.mark.gpu
def test_gpu_select_cursor_memory_is_bounded():
    """A ~10%-selective Select: the cursor keeps only the selected row ids (8 B each) plus one page
    -- no per-row expansion of the mask."""
    import torch

    ds = tpch.to_datasource(tpch.generate_flat(0.2, "cuda"), profile="bench")
    eng = Engine(use_native=True)
    q = S.SelectSpec("tpch", ["s_nation"], ["l_extendedprice"], filter=S.SelectorFilterSpec("s_region", "ASIA"),
                     intervals=["1992-01-01/1999-01-01"])
    pq = eng.prepare(q, ds)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    r = pq.run_page(S.PagingSpec({}, 10000))
    torch.cuda.synchronize()
    nsel = int(pq._sel_rows.numel())
    peak = torch.cuda.max_memory_allocated() - base
    assert r.num_rows == 10000 and nsel > 10 * 10000
    assert peak < 8 * nsel + ds.num_rows // 4 + (64 << 20), (peak, nsel)
    cpu = Engine(use_native=False).prepare(q, ds)
    ref = cpu.run_page(S.PagingSpec({}, 10000))
    assert np.array_equal(r.data["l_extendedprice"], ref.data["l_extendedprice"])
