"""The reference's BI plan (``docs/bi-benchmark/snap-sales-demo.jmx``) on the HIP engine, every one of
its 23 templates checked against the same SQL over the plain base table answered by the host pandas
operators (no lowering, no Druid rewrite shared: the reference's cTest pattern,
``tc/AbstractTest.scala:127-143``).  Three kernel paths:

* the JIT kernels (the serving default once a shape is compiled);
* the interpreter kernel (``ops/csrc/olap_scan.hip``) alone -- what a first-seen shape runs while its
  JIT source compiles in the background;
* the serving detour itself (``engine/device_exec.py async_compile``): cold code cache, first answer
  from the interim plan, second from the re-prepared JIT plan.
"""
import math

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import bi, tpch
from spark_druid_olap_amd.session import Session

pytestmark = pytest.mark.gpu

T = "orderLineItemPartSupplier"


@pytest.fixture(scope="module")
def bi_data():
    flat = tpch.generate_flat(0.05, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    df = tpch.to_pandas(flat)
    base = Session(engine=Engine(use_native=False))
    base.register_table("base", df, schema=tpch.FLAT_SCHEMA)
    bi.register(base, druid_table="base")
    # two "years" bindings per template (different literals, mostly the same kernel shapes)
    stmts = bi.statements(2, "years")
    exp = {q: _oracle(base, q) for _, _, q in stmts}
    return ds, stmts, exp


def _session(ds):
    s = Session(engine=Engine(use_native=True))
    s.register_datasource(ds)
    s.register_table(T + "Base", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    bi.register(s)
    return s


def _oracle(base, q):
    out = []
    for r in base.sql(q).to_pandas().itertuples(index=False, name=None):
        out.append(tuple(x.item() if hasattr(x, "item") else x for x in r))
    return out


def _rows(df):
    return [tuple(x.item() if hasattr(x, "item") else x for x in r)
            for r in df.to_pandas().itertuples(index=False, name=None)]


def _norm(v):
    import pandas as pd

    if v is None or v is pd.NA or v is pd.NaT:
        return None
    if isinstance(v, float):
        return None if math.isnan(v) else v
    return v


def _same(got, exp, q):
    assert len(got) == len(exp), (q, len(got), len(exp))
    key = lambda r: tuple((x is None, str(x)) for x in r)  # noqa: E731
    for a, b in zip(sorted(got, key=key), sorted(exp, key=key)):
        for x, y in zip(a, b):
            x, y = _norm(x), _norm(y)
            if isinstance(x, float) or isinstance(y, float):
                assert x is not None and y is not None and x == pytest.approx(y, rel=1e-6, abs=1e-6), (q, a, b)
            else:
                assert x == y, (q, a, b)


def _scans(df):
    from spark_druid_olap_amd.sql import plan as P

    out = []
    for dq in P.find_all_deep(df.plan, P.DruidQuery):
        prep = getattr(dq, "_prepared", None)
        out += [sc for _, _, sc in getattr(prep, "scans", []) if sc is not None]
    return out


@pytest.mark.timeout(600)
def test_bi_templates_jit_vs_base_table(bi_data):
    ds, stmts, exp = bi_data
    s = _session(ds)
    for name, _, q in stmts:
        d = s.sql(q)
        assert d.druid_queries(), (name, q)
        _same(_rows(d), exp[q], q)


@pytest.mark.timeout(600)
def test_bi_templates_interpreter_kernel_vs_base_table(bi_data, monkeypatch):
    """Every template on the interpreter kernel only (no JIT): the interim path of a first-seen
    shape while serving."""
    from spark_druid_olap_amd.engine import device_exec as DE

    monkeypatch.setattr(DE, "USE_JIT", False)
    ds, stmts, exp = bi_data
    s = _session(ds)
    ran = 0
    for name, _, q in stmts:
        d = s.sql(q)
        assert d.druid_queries(), (name, q)
        _same(_rows(d), exp[q], q)
        ran += sum(1 for sc in _scans(d) if sc.jit is None)
    assert ran > 0


@pytest.mark.timeout(900)
def test_bi_templates_async_compile_detour(bi_data, tmp_path, monkeypatch):
    """Cold code cache, first-seen shapes: each template's first answer comes from the interim plan
    (interpreter kernel where the scan allows it, background compiles pending), its second from the
    plan re-prepared once the compiles finished.  Both must equal the base-table answer."""
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.ops import jit

    monkeypatch.setenv("SDO_JIT_CACHE", str(tmp_path / "jit"))
    monkeypatch.setattr(jit, "_handles", {})
    monkeypatch.setattr(DE, "ASYNC_JIT", True)
    ds, stmts, exp = bi_data
    s = _session(ds)
    interim_scans = 0
    for name, _, q in stmts:
        d = s.sql(q)
        with DE.async_compile():
            d.prepare()
        from spark_druid_olap_amd.sql import plan as P

        pend = [f for dq in P.find_all_deep(d.plan, P.DruidQuery)
                for f in (getattr(getattr(dq, "_prepared", None), "jit_pending", None) or [])]
        interim_scans += sum(1 for sc in _scans(d) if sc.jit is None)
        _same(_rows(d), exp[q], q)
        for f in pend:
            f.result(timeout=300)
        d2 = s.sql(q)
        with DE.async_compile():
            d2.prepare()
        _same(_rows(d2), exp[q], q)
    assert interim_scans > 0


@pytest.mark.timeout(900)
def test_bi_templates_concurrent_serving_with_background_compiles(bi_data, tmp_path, monkeypatch):
    """The serving configuration that faulted in round 5 (64 BI clients, background compiles on):
    the native HiveServer2 gateway with its execution slots, a cold code cache, every first-seen
    shape on the interim interpreter plan while it compiles, re-prepared plans swapped in while
    other slots run.  16 clients run every statement in different orders; every answer must equal
    the base-table answer."""
    import threading

    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.ops import jit
    from spark_druid_olap_amd.server.gateway import NativeHiveServer
    from spark_druid_olap_amd.server.hive_client import connect

    monkeypatch.setenv("SDO_JIT_CACHE", str(tmp_path / "jit"))
    monkeypatch.setattr(jit, "_handles", {})
    monkeypatch.setattr(DE, "ASYNC_JIT", True)
    ds, stmts, exp = bi_data
    s = _session(ds)
    srv = NativeHiveServer(s, port=0)
    srv.start()
    errs, done = [], []
    try:
        def client(i):
            try:
                with connect(port=srv.port) as c:
                    order = stmts[i % len(stmts):] + stmts[:i % len(stmts)]
                    for _, _, q in (order if i % 2 else order[::-1]):
                        got = [tuple(r) for r in c.cursor().execute(q).fetchall()]
                        _same(got, exp[q], q)
                        done.append(q)
            except BaseException as e:  # noqa: BLE001
                errs.append(f"client {i}: {type(e).__name__}: {str(e)[:300]}")
        ts = [threading.Thread(target=client, args=(i,)) for i in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(800)
    finally:
        srv.stop()
    assert not errs, errs[:3]
    assert len(done) == 16 * len(stmts)
    from spark_druid_olap_amd.utils.metrics import events

    assert events().get("jit_async_interim", 0) > 0, events()
