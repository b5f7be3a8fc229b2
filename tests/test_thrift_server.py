"""HiveServer2 Thrift endpoint: SASL-PLAIN and noSasl clients, metadata calls, errors, concurrency
(the reference's HiveThriftServer2 entry point + JDBC clients)."""
import threading

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.server.hive_client import HiveError, connect
from spark_druid_olap_amd.server.hive_server import HiveThriftServer
from spark_druid_olap_amd.session import Session


@pytest.fixture(scope="module", params=["python", "native"])
def server(request, ds_small, df_small):
    """Every endpoint test runs against the pure-Python server and the native C++ gateway
    (server/csrc/hs2_gateway.cpp) in front of the same session."""
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    if request.param == "native":
        from spark_druid_olap_amd.server.gateway import NativeHiveServer

        srv = NativeHiveServer(s, port=0).start()
    else:
        srv = HiveThriftServer(s, port=0).start()
    yield srv
    srv.stop()


@pytest.mark.parametrize("sasl", [True, False])
def test_query_roundtrip(server, sasl, df_small):
    with connect(port=server.port, sasl=sasl) as c:
        cur = c.cursor().execute("select l_returnflag, count(*) c, sum(l_extendedprice) s "
                                 "from orderLineItemPartSupplier group by l_returnflag order by l_returnflag")
        assert cur.description == [("l_returnflag", "string"), ("c", "bigint"), ("s", "double")]
        rows = cur.fetchall()
        exp = df_small.groupby("l_returnflag").agg(c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"))
        assert [r[0] for r in rows] == list(exp.index)
        assert [r[1] for r in rows] == list(exp.c)
        for r, s in zip(rows, exp.s):
            assert r[2] == pytest.approx(s)
        cur.close()


def test_paging_nulls_and_errors(server):
    with connect(port=server.port) as c:
        cur = c.cursor()
        cur.arraysize = 7
        cur.execute("select o_orderkey, cast(null as string) n from orderLineItemPartSupplierBase limit 20")
        rows = cur.fetchall()
        assert len(rows) == 20 and all(r[1] is None for r in rows)
        with pytest.raises(HiveError):
            c.cursor().execute("select nosuchcol from orderLineItemPartSupplier")
        rows = c.cursor().execute("explain druid rewrite select count(*) from orderLineItemPartSupplier").fetchall()
        assert any("TimeSeriesQuerySpec" in r[0] for r in rows)


def test_metadata_calls(server):
    with connect(port=server.port) as c:
        r = c.call("GetTables", {"sessionHandle": c.session, "schemaName": "default", "tableName": "%"})
        cur = c.cursor()
        cur.op = r["operationHandle"]
        tabs = {row[2].lower() for row in cur.fetchall()}
        assert "orderlineitempartsupplier" in tabs
        r = c.call("GetColumns", {"sessionHandle": c.session, "tableName": "orderLineItemPartSupplier"})
        cur.op = r["operationHandle"]
        assert len(cur.fetchall()) == len(tpch.FLAT_SCHEMA)


def test_concurrent_clients(server):
    errs = []

    def client(i):
        try:
            with connect(port=server.port, sasl=bool(i % 2)) as c:
                for _ in range(3):
                    rows = c.cursor().execute("select s_region, count(*) from orderLineItemPartSupplier "
                                              "group by s_region").fetchall()
                    assert len(rows) == 5
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=client, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    if hasattr(server, "stats"):
        st = server.stats()
        # every statement went through the native path; batches <= statements
        assert st["statements"] >= 24 and st["batches"] <= st["statements"]


@pytest.mark.parametrize("coalesce", ["1", "0"])
def test_native_gateway_batches_identical_waiting_statements(ds_small, df_small, monkeypatch, coalesce):
    """With every executor busy, identical statements from different sessions that queue together
    execute once (one batch) and every client gets the full, correct result; a different statement
    is its own batch.  SDO_COALESCE=0 turns the sharing off: every statement is its own execution
    (what the concurrency benchmark's ``--coalesce off`` measures)."""
    import time as _t

    monkeypatch.setenv("SDO_COALESCE", coalesce)

    from spark_druid_olap_amd.server.gateway import NativeHiveServer

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    srv = NativeHiveServer(s, port=0, executors=1)
    gate = threading.Event()
    real = srv._execute

    def gated(bid, sid, stmt):
        if "s_region" in stmt:
            gate.wait(10)
        return real(bid, sid, stmt)

    srv._execute = gated
    srv.start()
    try:
        q_block = "select s_region, count(*) from orderLineItemPartSupplier group by s_region"
        q = "select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag order by l_returnflag"
        exp = [tuple(r) for r in df_small.groupby("l_returnflag").size().reset_index().itertuples(index=False)]
        outs, errs = [], []

        def run(sql, sink):
            try:
                with connect(port=srv.port) as c:
                    sink.append(c.cursor().execute(sql).fetchall())
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        blocker = threading.Thread(target=run, args=(q_block, []))
        blocker.start()
        _t.sleep(0.3)  # the only executor now holds the blocking batch
        ts = [threading.Thread(target=run, args=(q, outs)) for _ in range(6)]
        for t in ts:
            t.start()
        _t.sleep(0.5)
        before = srv.stats()
        gate.set()
        for t in ts + [blocker]:
            t.join(60)
        assert not errs, errs
        assert len(outs) == 6 and all([tuple(r) for r in o] == exp for o in outs)
        st = srv.stats()
        if coalesce == "1":
            assert before["coalesced"] >= 5 and st["batches"] == 2, (before, st)
        else:
            assert st["coalesced"] == 0 and st["batches"] == 7, (before, st)
    finally:
        srv.stop()


def test_native_gateway_new_statement_does_not_join_cancelled_batch(ds_small, df_small):
    """A queued batch whose only waiter cancelled keeps a sticky cancel flag; the same statement
    from another session must start a batch of its own and finish (it used to join the
    cancelled batch and fail with 'cancelled')."""
    import time as _t

    from spark_druid_olap_amd.server.gateway import NativeHiveServer

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    srv = NativeHiveServer(s, port=0, executors=1)
    gate = threading.Event()
    real = srv._execute

    def gated(bid, sid, stmt):
        if "s_region" in stmt:
            gate.wait(10)
        return real(bid, sid, stmt)

    srv._execute = gated
    srv.start()
    try:
        q_block = "select s_region, count(*) from orderLineItemPartSupplier group by s_region"
        q = "select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag order by l_returnflag"
        exp = [tuple(r) for r in df_small.groupby("l_returnflag").size().reset_index().itertuples(index=False)]
        blocker = threading.Thread(target=lambda: connect(port=srv.port).cursor().execute(q_block).fetchall())
        blocker.start()
        _t.sleep(0.3)  # the only executor now holds the blocking batch: q stays queued
        with connect(port=srv.port) as a, connect(port=srv.port) as b:
            r = a.call("ExecuteStatement", {"sessionHandle": a.session, "statement": q, "runAsync": True})
            a.call("CancelOperation", {"operationHandle": r["operationHandle"]})
            out = []
            t = threading.Thread(target=lambda: out.append(b.cursor().execute(q).fetchall()))
            t.start()
            _t.sleep(0.3)
            gate.set()
            t.join(60)
            blocker.join(60)
            assert out and [tuple(x) for x in out[0]] == exp
    finally:
        gate.set()
        srv.stop()


def test_sessions_do_not_share_set_or_use(server):
    """Per-client session state (Session.new_session): SET and USE in one client session are not
    seen by another; tables stay shared."""
    srv_sess = server.session
    srv_sess.sql("create database if not exists other_db")
    with connect(port=server.port) as a, connect(port=server.port) as b:
        a.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize=17")
        a.cursor().execute("use other_db")
        got_a = a.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize").fetchall()
        got_b = b.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize").fetchall()
        assert got_a[0][1] == "17" and got_b[0][1] != "17"
        # b still resolves unqualified names in `default`; a needs the qualified name now
        assert b.cursor().execute("select count(*) from orderLineItemPartSupplier").fetchall()[0][0] > 0
        with pytest.raises(HiveError):
            a.cursor().execute("select count(*) from orderLineItemPartSupplier")
        assert a.cursor().execute("select count(*) from default.orderLineItemPartSupplier").fetchall()[0][0] > 0
    assert srv_sess.catalog.current_db == "default"
    assert srv_sess.conf.get("spark.sparklinedata.druid.selectquery.pagesize") != "17"


def test_identical_queued_statements_execute_once():
    """engine/scheduler.py: with one stream slot busy, identical statements that queue up together
    run once and every waiter gets the result."""
    import time as _t

    from spark_druid_olap_amd.engine.scheduler import Coalescer, StreamScheduler

    co = Coalescer(StreamScheduler(1))
    calls = []
    gate = threading.Event()

    def slow():
        calls.append(1)
        gate.wait(5)
        return len(calls)

    blocker = threading.Thread(target=lambda: co.run("other", slow))
    blocker.start()
    _t.sleep(0.1)  # the only slot is now held
    outs = []
    ts = [threading.Thread(target=lambda: outs.append(co.run("q", lambda: (calls.append(2), "r")[1])))
          for _ in range(5)]
    for t in ts:
        t.start()
    _t.sleep(0.2)
    gate.set()
    for t in ts + [blocker]:
        t.join(10)
    assert outs == ["r"] * 5
    assert calls.count(2) == 1 and co.stats["coalesced"] == 4


@pytest.mark.timeout(300)
def test_two_rank_server_returns_merged_answer(tmp_path):
    """HiveServer2 over all ranks (server/spmd.py): ``--gpus 2`` starts two ranks (gloo on CPU),
    each holding its own TPC-H shard; a client of rank 0 gets the answer over the union of both
    shards, and SET in its session travels to the peer."""
    import os
    import signal
    import subprocess
    import sys
    import time as _t

    import pandas as pd

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pf = tmp_path / "port"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", PYTHONPATH=root)
    p = subprocess.Popen([sys.executable, "-m", "spark_druid_olap_amd.server.hive_server", "--gpus", "2",
                          "--tpch-sf", "0.003", "--port", "0", "--port-file", str(pf), "--ui-port", "-1"],
                         cwd=root, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        t0 = _t.time()
        while not pf.exists():
            assert p.poll() is None, p.stderr.read().decode()[-3000:]
            assert _t.time() - t0 < 200, "server did not start"
            _t.sleep(0.2)
        port = int(pf.read_text())
        full = pd.concat([tpch.to_pandas(tpch.generate_flat(0.003, "cpu", rank=r, world=2)) for r in range(2)])
        exp = full.groupby("l_returnflag").agg(c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"))
        q = ("select l_returnflag, count(*) c, sum(l_extendedprice) s from orderLineItemPartSupplier "
             "group by l_returnflag order by l_returnflag")
        with connect(port=port) as c1, connect(port=port) as c2:
            for c in (c1, c2):
                rows = c.cursor().execute(q).fetchall()
                assert [r[0] for r in rows] == list(exp.index)
                assert [r[1] for r in rows] == list(exp.c)
                for r, s in zip(rows, exp.s):
                    assert r[2] == pytest.approx(s)
            c1.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize=5")
            assert c1.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize").fetchall()[0][1] == "5"
            n = c2.cursor().execute("select count(distinct o_orderkey) from orderLineItemPartSupplier").fetchall()
            assert n[0][0] == full.o_orderkey.nunique()
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(60)
        except subprocess.TimeoutExpired:
            p.kill()
    assert p.returncode == 0, p.stderr.read().decode()[-3000:]


def test_two_rank_python_server_streams_select_pages(tmp_path):
    """A Select-backed statement on the multi-rank Python server pages through a cursor that every
    rank advances on the same broadcast message (server/spmd.py streams): the client gets every
    row of both shards, a page at a time (page size 7)."""
    import os
    import signal
    import subprocess
    import sys
    import time as _t

    import pandas as pd

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pf = tmp_path / "port"
    init = tmp_path / "init.sql"
    # a second table over the same index whose plain selects push down as Druid Select queries
    init.write_text(tpch.druid_ddl(table="lineitemSelect", with_column_mapping=False,
                                   star_schema='{"factTable" : "lineitemSelect", "relations" : []}',
                                   extra_options=', nonAggregateQueryHandling "push_project_and_filters"'))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", PYTHONPATH=root, SDO_NATIVE_GATEWAY="0", SDO_STREAM_MIN_GROUPS="1000")
    p = subprocess.Popen([sys.executable, "-m", "spark_druid_olap_amd.server.hive_server", "--gpus", "2",
                          "--tpch-sf", "0.002", "--port", "0", "--port-file", str(pf), "--ui-port", "-1",
                          "--init-sql", str(init)],
                         cwd=root, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        t0 = _t.time()
        while not pf.exists():
            assert p.poll() is None, p.stderr.read().decode()[-3000:]
            assert _t.time() - t0 < 200, "server did not start"
            _t.sleep(0.2)
        port = int(pf.read_text())
        full = pd.concat([tpch.to_pandas(tpch.generate_flat(0.002, "cpu", rank=r, world=2)) for r in range(2)])
        want = sorted(zip(full[full.l_returnflag == "R"].o_orderkey, full[full.l_returnflag == "R"].l_quantity))
        with connect(port=port) as c:
            c.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize=7")
            cur = c.cursor().execute("select o_orderkey, l_quantity from lineitemSelect where l_returnflag = 'R'")
            got = sorted((int(a), int(b)) for a, b in cur.fetchall())
            assert got == [(int(a), int(b)) for a, b in want]
            # a cursor closed before its end releases the stream on every rank; the server goes on
            cur = c.cursor().execute("select o_orderkey from lineitemSelect")
            cur.close()
            n = c.cursor().execute("select count(*) from orderLineItemPartSupplier").fetchall()[0][0]
            assert n == len(full)
            # a large groupBy streams too: rank 0 pages through the gathered groups
            c.cursor().execute("set spark.sparklinedata.druid.selectquery.pagesize=997")
            cur = c.cursor().execute("select o_orderkey, l_linenumber, count(*) from orderLineItemPartSupplier "
                                     "group by o_orderkey, l_linenumber")
            got = sorted((int(a), int(b), int(n_)) for a, b, n_ in cur.fetchall())
            exp = full.groupby(["o_orderkey", "l_linenumber"]).size()
            assert got == sorted((int(a), int(b), int(v)) for (a, b), v in exp.items())
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(60)
        except subprocess.TimeoutExpired:
            p.kill()
    assert p.returncode == 0, p.stderr.read().decode()[-3000:]


def test_warm_up_runs_each_statement_on_a_slot(ds_small, df_small):
    """server/gateway.py warm_up: statements run on leased execution slots (commands just execute)
    and the call reports what it ran; without a GPU the device-memory sizing is a no-op."""
    from spark_druid_olap_amd.server.gateway import warm_up

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    leases0 = s.engine.coalescer().scheduler.stats["leases"]
    out = warm_up(s, ["select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag",
                      "set spark.sparklinedata.druid.deterministic=false"])
    assert out["statements_run"] == 1
    assert s.engine.coalescer().scheduler.stats["leases"] == leases0 + 1
