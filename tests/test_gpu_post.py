"""GPU: the fused post-scan path and an engine-independent oracle.

* ``native.touch_compact`` (post_scan.hip touch_*) against a plain torch compaction of the same
  first-touch table: ids, gathered rows, re-initialised rows and cleared bytes;
* the sparse finalize kernel (post_scan.hip sparse_decode_kernel) against the torch finalize
  path on SQL queries with typed / FD-derived keys and every aggregator output kind;
* the 8 headline SQL queries through the HIP engine checked against pandas on the generated rows
  (the reference's cTest oracle over base tables, tc/AbstractTest.scala:127-143) -- a lowering
  bug shared by the HIP kernels and the torch reference executor cannot pass this one.
"""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def flat_gpu():
    from spark_druid_olap_amd.models import tpch

    return tpch.generate_flat(0.05, "cuda")


@pytest.fixture(scope="module")
def sess(flat_gpu):
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    ds = tpch.to_datasource(flat_gpu, profile="bench")
    s = Session(engine=Engine(), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    return s


@pytest.fixture(scope="module")
def df(flat_gpu):
    from spark_druid_olap_amd.models import tpch

    return tpch.to_pandas(flat_gpu)


def test_touch_compact_matches_torch():
    from spark_druid_olap_amd.ops import native

    g = torch.Generator(device="cuda").manual_seed(7)
    for rows in (1, 63, 64, 65, 100_003, (1 << 20) + 17):
        ns = 3
        touch = torch.zeros((rows + 63) // 64 * 64, dtype=torch.uint8, device="cuda")
        sel = torch.rand(rows, generator=g, device="cuda") < 0.07
        touch[:rows][sel] = 1
        acc = torch.randint(-1000, 1000, (rows, ns), generator=g, device="cuda", dtype=torch.int64)
        before = acc.clone()
        init = torch.tensor([0, 1 << 40, -(1 << 40)], dtype=torch.int64, device="cuda")
        idx, out = native.touch_compact(touch, acc, init)
        ref = torch.nonzero(sel).flatten()
        assert torch.equal(idx, ref), rows
        assert torch.equal(out, before[ref])
        assert torch.equal(acc[ref], init.expand(ref.numel(), -1))
        keep = ~sel
        assert torch.equal(acc[keep], before[keep])
        assert int(touch.sum()) == 0
        idx2, out2 = native.touch_compact(touch, acc, init)  # nothing touched now
        assert idx2.numel() == 0 and out2.shape == (0, ns)


DECODE_SQL = [
    # TPC-H Q3 of the benchmark: range-typed o_orderkey, FD-derived o_orderdate / o_shippriority
    """select o_orderkey, sum(l_extendedprice) as price, o_orderdate, o_shippriority
       from orderLineItemPartSupplier where c_mktsegment = 'BUILDING'
         and dateIsBefore(dateTime(`o_orderdate`), dateTime("1995-03-15"))
         and dateIsAfter(dateTime(`l_shipdate`), dateTime("1995-03-15"))
       group by o_orderkey, o_orderdate, o_shippriority""",
    # counts, long sums, float min / max, averages over a large key space
    """select o_orderkey, l_linenumber, count(*) as c, sum(l_quantity) as q, min(l_extendedprice) as mn,
              max(l_discount) as mx, avg(l_tax) as t
       from orderLineItemPartSupplier where l_shipmode = 'AIR' group by o_orderkey, l_linenumber""",
    """select c_name, p_brand, sum(l_extendedprice) as s, count(*) as c from orderLineItemPartSupplier
       where o_orderdate >= '1996-01-01' group by c_name, p_brand""",
]


@pytest.mark.parametrize("qi", range(len(DECODE_SQL)))
def test_sparse_decode_kernel_matches_torch_finalize(sess, qi, monkeypatch):
    from spark_druid_olap_amd.engine import partials as P

    q = DECODE_SQL[qi]
    calls = []
    real = P._native_sparse

    def spy(*a, **k):
        r = real(*a, **k)
        calls.append(r is not None)
        return r

    monkeypatch.setattr(P, "_native_sparse", spy)
    monkeypatch.setattr(P, "SMALL_DENSE_WORDS", 0)  # small dense tables too take the sparse path
    got = sess.sql(q).to_pandas()
    assert any(calls), "the native sparse decode did not run"
    monkeypatch.setattr(P, "NATIVE_DECODE", False)
    sess._plan_cache.clear()
    ref = sess.sql(q).to_pandas()
    assert len(got) > 100 and list(got.columns) == list(ref.columns)
    cols = list(got.columns)
    a = got.sort_values(cols).reset_index(drop=True)
    b = ref.sort_values(cols).reset_index(drop=True)
    for c in cols:
        assert a[c].dtype == b[c].dtype, c
        if a[c].dtype.kind == "f":  # (float sums: device atomics add in a different order per run)
            np.testing.assert_allclose(a[c].to_numpy(), b[c].to_numpy(), rtol=1e-12)
        else:
            assert a[c].tolist() == b[c].tolist(), c


def _ship(d):
    return (d.l_shipdate > "1995-12-01") & (d.l_shipdate <= "1997-09-02")


def _nations(d):
    return ((d.s_nation == "FRANCE") & (d.c_nation == "GERMANY")) | ((d.c_nation == "FRANCE") & (d.s_nation == "GERMANY"))


def _rows(frame, keys):
    return {tuple(r[:len(keys)]): tuple(r[len(keys):]) for r in frame.itertuples(index=False, name=None)}


def test_headline_queries_match_pandas(sess, df):
    """The 8 headline SQL statements on the HIP engine vs pandas over the generated rows."""
    from spark_druid_olap_amd.models import tpch

    qs = dict(tpch.BENCH_QUERIES)

    def check(name, frame, keys, aggs, tol=1e-9):
        got = sess.sql(qs[name]).to_pandas()
        exp = frame.groupby(keys).agg(**aggs).reset_index() if keys else \
            pd.DataFrame({k: [v[1](frame[v[0]])] for k, v in aggs.items()})
        assert len(got) == len(exp), name
        gk = [c for c in got.columns][:len(keys)]
        g = {tuple(str(x) for x in r[:len(keys)]): r[len(keys):] for r in got.itertuples(index=False, name=None)}
        for r in exp.itertuples(index=False, name=None):
            k, v = tuple(str(x) for x in r[:len(keys)]), r[len(keys):]
            assert k in g, (name, k, gk)
            for x, y in zip(g[k], v):
                assert x == pytest.approx(y, rel=tol), (name, k, x, y)

    d = df
    q1 = dict(c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"), m=("ps_supplycost", "max"),
              a=("ps_availqty", "mean"))
    for name in ("Basic Aggregation", "TPCH Q1"):
        got = sess.sql(qs[name]).to_pandas()
        exp = d.groupby(["l_returnflag", "l_linestatus"]).agg(**q1, n=("o_orderkey", "nunique")).reset_index()
        g = _rows(got, ["f", "s"])
        assert len(g) == len(exp)
        for r in exp.itertuples(index=False, name=None):
            v = g[(r[0], r[1])]
            assert v[0] == r[2] and v[1] == pytest.approx(r[3], rel=1e-9) and v[2] == pytest.approx(r[4])
            assert v[3] == pytest.approx(r[5], rel=1e-9)
            assert v[4] == pytest.approx(r[6], rel=0.08)  # HLL p=11
    check("Ship Date Range", d[_ship(d)], ["l_returnflag", "l_linestatus"], dict(c=("l_shipdate", "size")))
    sub = d[_ship(d) & (d.p_type == "ECONOMY ANODIZED STEEL") & _nations(d)]
    got = sess.sql(qs["SubQuery + nation,Type predicates + ShipDate Range"]).to_pandas()
    exp = sub.groupby("s_nation").agg(c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"),
                                      m=("ps_supplycost", "max"), a=("ps_availqty", "mean"))
    g = _rows(got, ["s_nation"])
    assert set(g) == {(k,) for k in exp.index}
    for k, r in exp.iterrows():
        v = g[(k,)]
        assert v[0] == r.c and v[1] == pytest.approx(r.s, rel=1e-9) and v[2] == pytest.approx(r.m)
        assert v[3] == pytest.approx(r.a, rel=1e-9)
    sub = d[(d.c_mktsegment == "BUILDING") & (d.o_orderdate < "1995-03-15") & (d.l_shipdate > "1995-03-15")]
    got = sess.sql(qs["TPCH Q3"]).to_pandas()
    exp = sub.groupby(["o_orderkey", "o_orderdate", "o_shippriority"]).l_extendedprice.sum()
    assert len(got) == len(exp) > 100
    gq = {(int(a), str(c), int(e)): b for a, b, c, e in got.itertuples(index=False, name=None)}
    for (a, c, e), v in exp.items():
        assert gq[(int(a), str(c), int(e))] == pytest.approx(v, rel=1e-9)
    check("TPCH Q5", d[(d.s_region == "ASIA") & (d.o_orderdate >= "1994-01-01") & (d.o_orderdate < "1995-01-01")],
          ["s_nation"], dict(s=("l_extendedprice", "sum")))
    sub = d[_nations(d)]
    check("TPCH Q7", sub.assign(y=sub.l_shipdate.str[:4]), ["s_nation", "c_nation", "y"],
          dict(s=("l_extendedprice", "sum")))
    sub = d[(d.c_region == "AMERICA") & (d.p_type == "ECONOMY ANODIZED STEEL") & (d.o_orderdate >= "1995-01-01")
            & (d.o_orderdate <= "1996-12-31")]
    check("TPCH Q8", sub.assign(y=sub.o_orderdate.str[:4]), ["y"], dict(s=("l_extendedprice", "sum")))


def test_device_lexsort_equals_numpy():
    """sql/execute.py sort_indices on the GPU (large host sorts: ORDER BY, window partitions) is
    np.lexsort exactly -- ties keep row order, nulls and DESC folded as on the host."""
    from spark_druid_olap_amd.sql import execute as X

    rng = np.random.default_rng(5)
    n = 200_003
    lex = [rng.integers(0, 50, n), rng.normal(size=n).round(2), rng.integers(0, 7, n).astype(np.int64),
           rng.random(n) < 0.1]
    assert np.array_equal(X._lexsort_device(lex), np.lexsort(lex))
    s = pd.Series(rng.integers(0, 100, n).astype(float))
    s[rng.random(n) < 0.05] = np.nan
    keys = [(pd.Series(rng.integers(0, 9, n)), True, None), (s, False, None)]
    dev = X.sort_indices(keys, n)
    X.GPU_SORT_MIN_ROWS, old = 1 << 40, X.GPU_SORT_MIN_ROWS
    try:
        host = X.sort_indices(keys, n)
    finally:
        X.GPU_SORT_MIN_ROWS = old
    assert np.array_equal(dev, host)
