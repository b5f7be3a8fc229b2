"""CPU engine tests: torch reference executor vs a pandas oracle on the same synthetic TPC-H shard
(the reference's cTest strategy, tc/AbstractTest.scala:127-143, with pandas in Spark's role)."""
import glob
import json
import os

import numpy as np
import pandas as pd
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models.bench_queries import bench_specs
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.query.spec import query_from_json

REF_Q = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "parity", "benchmark_queries", "*.json")))


def run(q, ds):
    return Engine(use_native=False).execute(q, ds)


def _nation_pair(df):
    return (((df.s_nation == "FRANCE") & (df.c_nation == "GERMANY")) |
            ((df.c_nation == "FRANCE") & (df.s_nation == "GERMANY")))


def _ship_range(df):
    return (df.l_shipdate > "1995-12-01") & (df.l_shipdate <= "1997-09-02")


def test_q1_matches_pandas(ds_small, df_small):
    r = run(dict(bench_specs())["TPCH Q1"], ds_small)
    g = df_small.groupby(["l_returnflag", "l_linestatus"]).agg(
        c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"), m=("ps_supplycost", "max"),
        a=("ps_availqty", "sum"), d=("o_orderkey", "nunique")).reset_index()
    got = r.to_pandas().sort_values(["l_returnflag", "l_linestatus"]).reset_index(drop=True)
    assert len(got) == len(g)
    np.testing.assert_array_equal(got["alias-1"], g.c)
    np.testing.assert_allclose(got["alias-2"], g.s, rtol=1e-12)
    np.testing.assert_allclose(got["alias-3"], g.m)
    np.testing.assert_array_equal(got["alias-5"], g.a)
    np.testing.assert_allclose(got["alias-4"], g.a / g.c)
    # HyperLogLog p=11: ~2.3% standard error
    np.testing.assert_allclose(got["alias-7"], g.d, rtol=0.08)


def test_ship_date_range(ds_small, df_small):
    r = run(dict(bench_specs())["Ship Date Range"], ds_small)
    sub = df_small[_ship_range(df_small)]
    g = sub.groupby(["l_returnflag", "l_linestatus"]).size()
    got = {(a, b): c for a, b, c in r.rows()}
    assert got == {k: int(v) for k, v in g.items()}


def test_projfiltrange(ds_small, df_small):
    r = run(dict(bench_specs())["SubQuery + nation,Type predicates + ShipDate Range"], ds_small)
    sub = df_small[_ship_range(df_small) & (df_small.p_type == "ECONOMY ANODIZED STEEL") & _nation_pair(df_small)]
    g = sub.groupby("s_nation").l_extendedprice.sum()
    got = {row[0]: row[2] for row in r.rows()}
    assert set(got) == set(g.index)
    for k in got:
        assert got[k] == pytest.approx(g[k])


def test_q3_q5_q7_q8(ds_small, df_small):
    specs = dict(bench_specs())
    df = df_small
    r3 = run(specs["TPCH Q3"], ds_small)
    sub = df[(df.c_mktsegment == "BUILDING") & (df.o_orderdate < "1995-03-15") & (df.l_shipdate > "1995-03-15")]
    g3 = sub.groupby(["o_orderkey", "o_orderdate", "o_shippriority"]).l_extendedprice.sum()
    assert r3.num_rows == len(g3)
    got3 = {(a, b, c): v for a, b, c, v in r3.rows()}
    for k, v in g3.items():
        assert got3[k] == pytest.approx(v)
    r5 = run(specs["TPCH Q5"], ds_small)
    sub = df[(df.s_region == "ASIA") & (df.o_orderdate >= "1994-01-01") & (df.o_orderdate < "1995-01-01")]
    g5 = sub.groupby("s_nation").l_extendedprice.sum()
    assert {a: pytest.approx(b) for a, b in r5.rows()} == {k: pytest.approx(v) for k, v in g5.items()}
    r7 = run(specs["TPCH Q7"], ds_small)
    sub = df[_nation_pair(df)]
    g7 = sub.assign(y=sub.l_shipdate.str[:4]).groupby(["s_nation", "c_nation", "y"]).l_extendedprice.sum()
    assert {(a, b, c): pytest.approx(v) for a, b, c, v in r7.rows()} == {k: pytest.approx(v) for k, v in g7.items()}
    r8 = run(specs["TPCH Q8"], ds_small)
    sub = df[(df.c_region == "AMERICA") & (df.p_type == "ECONOMY ANODIZED STEEL") & (df.o_orderdate >= "1995-01-01")
             & (df.o_orderdate <= "1996-12-31")]
    g8 = sub.assign(y=sub.o_orderdate.str[:4]).groupby("y").l_extendedprice.sum()
    assert {a: pytest.approx(b) for a, b in r8.rows()} == {k: pytest.approx(v) for k, v in g8.items()}


def test_filters_expressions_filtered_aggs(ds_small, df_small):
    types = ["ECONOMY ANODIZED STEEL", "PROMO BRUSHED TIN", "SMALL PLATED COPPER", "LARGE BURNISHED NICKEL",
             "MEDIUM POLISHED BRASS", "STANDARD ANODIZED TIN"]
    f = S.LogicalFilterSpec("and", [
        S.InFilterSpec("p_type", types), S.NotFilterSpec(S.SelectorFilterSpec("l_shipmode", "AIR")),
        S.BoundFilterSpec("o_orderdate", "1993-01-01", "1996-06-30", False, True),
        S.BoundFilterSpec("l_quantity", "5", "45", True, False)])
    aggs = [S.FunctionAggregationSpec("count", "c"), S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice"),
            S.JavascriptAggregationSpec("rev", ["l_extendedprice", "l_discount"],
                                        "function(current, a, b) { return current + (a * (1 - b)); }",
                                        "function(a,b){return a+b;}", "function(){return 0;}"),
            S.FilteredAggregationSpec(S.SelectorFilterSpec("l_returnflag", "R"),
                                      S.FunctionAggregationSpec("longSum", "q_r", "l_quantity"), "q_r")]
    q = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("c_region"), S.DefaultDimensionSpec("l_linestatus")],
                           filter=f, aggregations=aggs, intervals=["1992-01-01/1999-01-01"])
    r = run(q, ds_small).to_pandas().sort_values(["c_region", "l_linestatus"]).reset_index(drop=True)
    df = df_small
    m = (df.p_type.isin(types) & (df.l_shipmode != "AIR") & (df.o_orderdate >= "1993-01-01") &
         (df.o_orderdate < "1996-06-30") & (df.l_quantity > 5) & (df.l_quantity <= 45))
    sub = df[m].assign(rev=lambda x: x.l_extendedprice * (1 - x.l_discount),
                       qr=lambda x: np.where(x.l_returnflag == "R", x.l_quantity, 0))
    g = sub.groupby(["c_region", "l_linestatus"]).agg(c=("rev", "size"), s=("l_extendedprice", "sum"),
                                                      rev=("rev", "sum"), qr=("qr", "sum")).reset_index()
    np.testing.assert_array_equal(r.c, g.c)
    np.testing.assert_allclose(r.s, g.s)
    np.testing.assert_allclose(r.rev, g.rev)
    np.testing.assert_array_equal(r.q_r, g.qr)


def test_timeseries_topn_search_select(ds_small, df_small):
    q = S.TimeSeriesQuerySpec("tpch", ["1994-01-01/1996-01-01"], granularity=S.Granularity.parse("month"),
                              aggregations=[S.FunctionAggregationSpec("longSum", "q", "l_quantity")])
    r = run(q, ds_small)
    assert r.num_rows == 24
    sub = df_small[(df_small.l_shipdate >= "1994-01-01") & (df_small.l_shipdate < "1996-01-01")]
    assert int(r.data["q"].sum()) == int(sub.l_quantity.sum())
    t = S.TopNQuerySpec("tpch", S.DefaultDimensionSpec("p_brand"), S.NumericTopNMetricSpec("s"), 5,
                        ["1992-01-01/1999-01-01"], aggregations=[S.FunctionAggregationSpec("doubleSum", "s",
                                                                                         "l_extendedprice")])
    r = run(t, ds_small)
    want = df_small.groupby("p_brand").l_extendedprice.sum().sort_values(ascending=False).head(5)
    assert [row[0] for row in r.rows()] == list(want.index)
    sq = S.SearchQuerySpec("tpch", ["1992-01-01/1999-01-01"], searchDimensions=["c_nation", "s_nation"],
                           query=S.SearchQueryQuerySpec("insensitive_contains", "an"))
    r = run(sq, ds_small)
    vals = set(r.data["value"].tolist())
    assert "JAPAN" in vals and "FRANCE" in vals and "CHINA" not in vals
    assert r.data["dimension"].tolist().count("c_nation") == len([v for v in df_small.c_nation.unique() if "an" in v.lower()])
    sel = S.SelectSpec("tpch", ["s_nation"], ["l_extendedprice"],
                       filter=S.SelectorFilterSpec("s_nation", "FRANCE"), pagingSpec=S.PagingSpec({}, 7),
                       intervals=["1992-01-01/1999-01-01"])
    r1 = run(sel, ds_small)
    assert r1.num_rows == 7 and set(r1.data["s_nation"].tolist()) == {"FRANCE"}
    sel2 = sel.copy(pagingSpec=S.PagingSpec(r1.paging, 7))
    r2 = run(sel2, ds_small)
    assert r2.data["timestamp"][0] >= r1.data["timestamp"][-1]


def test_having_limit_postagg(ds_small):
    q = S.GroupByQuerySpec(
        "tpch", [S.DefaultDimensionSpec("s_nation")],
        aggregations=[S.FunctionAggregationSpec("count", "c"), S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice")],
        postAggregations=[S.ArithmeticPostAggregationSpec("/", [S.FieldAccessPostAggregationSpec("s"),
                                                               S.FieldAccessPostAggregationSpec("c")], "avg")],
        having=S.ComparisonHavingSpec("greaterThan", "c", 100),
        limitSpec=S.LimitSpec(3, [S.OrderByColumnSpec("avg", "descending")]),
        intervals=["1992-01-01/1999-01-01"])
    r = run(q, ds_small)
    assert r.num_rows == 3
    avg = r.data["avg"]
    assert list(avg) == sorted(avg, reverse=True)
    assert all(c > 100 for c in r.data["c"])


@pytest.mark.skipif(not REF_Q, reason="reference checkout not mounted")
@pytest.mark.parametrize("path", REF_Q)
def test_reference_json_roundtrip_and_executes(path, ds_small):
    d = json.load(open(path))
    q = query_from_json(d)

    def strip(x):
        if isinstance(x, dict):
            return {k: strip(v) for k, v in x.items()}
        if isinstance(x, list):
            return [strip(v) for v in x]
        return x

    assert strip(q.to_json()) == strip(d)
    r = run(q, ds_small)
    assert r.num_rows >= 1


def test_dimension_lut_aggregators(ds_small, df_small):
    """Dimensions in row expressions read their dictionary entries as numbers (E_LUT);
    longMin/longMax over __time."""
    import numpy as np

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.query import spec as S

    aggs = [S.JavascriptAggregationSpec("s_ln", ["l_linenumber"], "function(current, a) { return current + a; }",
                                        "function(a,b){return a+b;}", "function(){return 0;}"),
            S.JavascriptAggregationSpec("mn_od", ["o_orderdate"], "function(current, a) { return Math.min(current, a); }",
                                        "function(a,b){return Math.min(a,b);}", "function(){return Infinity;}"),
            S.FunctionAggregationSpec("longMin", "t0", "__time"),
            S.FunctionAggregationSpec("longMax", "t1", "__time")]
    q = S.TimeSeriesQuerySpec("tpch", ["1992-01-01/1999-01-01"], aggregations=aggs)
    r = Engine(use_native=False).execute(q, ds_small)
    assert int(r.data["s_ln"][0]) == int(df_small["l_linenumber"].sum())
    od = pd_ms(df_small["o_orderdate"].min())
    assert int(r.data["mn_od"][0]) == od
    assert int(r.data["t0"][0]) == pd_ms(df_small["l_shipdate"].min())
    assert int(r.data["t1"][0]) == pd_ms(df_small["l_shipdate"].max())


def pd_ms(s):
    import pandas as pd

    return int(pd.Timestamp(s).value // 1_000_000)


@pytest.mark.parametrize("direction,metric", [("descending", "p"), ("ascending", "p"), ("descending", "c")])
def test_device_topk_prune_matches_full_sort(ds_small, direction, metric):
    """ORDER BY <aggregate> LIMIT k prunes the merged partials on the device (ties at the k-th value
    kept) and must equal sorting every group."""
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.query import spec as S

    dims = [S.DefaultDimensionSpec("o_orderkey")]
    aggs = [S.FunctionAggregationSpec("doubleSum", "p", "l_extendedprice"), S.FunctionAggregationSpec("count", "c")]
    ls = S.LimitSpec(25, [S.OrderByColumnSpec("p" if metric == "p" else "c", direction),
                          S.OrderByColumnSpec("o_orderkey", "ascending")])
    q = S.GroupByQuerySpec("tpch", dims, aggregations=aggs, intervals=["1992-01-01/1999-01-01"], limitSpec=ls)
    full = Engine(use_native=False).execute(q.copy(limitSpec=None), ds_small)
    assert full.num_rows > 4096
    got = Engine(use_native=False).execute(q, ds_small)
    rows = full.rows()
    m = 1 if metric == "p" else 2
    sign = -1 if direction == "descending" else 1
    rows.sort(key=lambda r: (sign * r[m], r[0]))
    assert got.rows() == rows[:25]


def test_scan_buffer_budget_releases_least_recently_used(monkeypatch):
    """Cached plans keep their programs, but per-slot device buffers beyond the budget are released
    LRU-first (engine/device_exec.py); a released scan re-allocates on its next run."""
    import threading

    import torch

    from spark_druid_olap_amd.engine import device_exec as DE

    class Prep:
        def __init__(self):
            self._slots, self._slot_lock = {}, threading.Lock()

    def bufs(n):
        b = DE._Bufs()
        b.acc, b.keys, b.overflow, b.desc = torch.zeros(n, dtype=torch.int64), torch.zeros(1), torch.zeros(1), \
            torch.zeros(1)
        b.touch, b.init_row, b.hll, b.hll32, b.part = torch.zeros(1), torch.zeros(1), [], [], None
        return b

    monkeypatch.setattr(DE, "BUF_BUDGET", 28_000)
    preps = [Prep() for _ in range(4)]
    for p in preps:
        p._slots[0] = bufs(1000)
        DE._buffers_acquired(p, 0, p._slots[0])
    # ~8 KB each against a 24 KB budget: the oldest went
    assert not preps[0]._slots and all(p._slots for p in preps[1:])
    DE._buffers_used(preps[1], 0)          # touched: now the most recent
    preps[0]._slots[0] = bufs(1000)
    DE._buffers_acquired(preps[0], 0, preps[0]._slots[0])
    assert preps[1]._slots and not preps[2]._slots
    for p in preps:
        DE._forget_prep(id(p))
    assert DE._buf_total[0] >= 0
