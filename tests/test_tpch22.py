"""TPC-H 22-query sweep (BASELINE config 2) over the flattened orderLineItemPartSupplier index.

Every query must push its row-level work to the engine (at least one Druid query, scalar
subqueries included) and return the same rows as the identical SQL over the plain base table
(the reference's cTest pattern, ``tc/AbstractTest.scala:127-143``).  CPU: torch reference
executor.  The GPU twin (tests/test_gpu_tpch22.py) compares the HIP kernels with it."""
import math

import numpy as np
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch, tpch22
from spark_druid_olap_amd.segment.dictionary import WordsDictionary
from spark_druid_olap_amd.session import Session

T = "orderLineItemPartSupplier"
B = "orderLineItemPartSupplierBase"


@pytest.fixture(scope="module")
def sess(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table(B, df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s


def _norm(v):
    if isinstance(v, float):
        return None if math.isnan(v) else round(v, 2)
    return v


def _rows(d):
    return sorted((tuple(_norm(v) for v in r) for r in d.collect()), key=lambda r: tuple((x is None, str(x)) for x in r))


@pytest.mark.parametrize("name", [n for n, _ in tpch22.QUERIES])
def test_tpch22_pushed_and_exact(sess, name):
    q = dict(tpch22.QUERIES)[name]
    d = sess.sql(q)
    assert d.druid_queries(), d.explain()
    got = _rows(d)
    exp = _rows(sess.sql(q.replace(T, B)))
    assert len(got) == len(exp), (len(got), len(exp))
    for x, y in zip(got, exp):
        for a, c in zip(x, y):
            if isinstance(a, float) or isinstance(c, float):
                assert a == pytest.approx(c, rel=1e-6, abs=0.02), (x, y)
            else:
                assert a == c, (x, y)


def test_tpch22_non_trivial_answers(sess):
    """The LIKE-driven queries (part colours, comment text) select real rows on synthetic data."""
    for name in ("Q9", "Q13", "Q16", "Q20"):
        assert len(sess.sql(dict(tpch22.QUERIES)[name]).collect()) > 0, name


def test_scalar_subquery_filter_is_deferred(sess):
    q = dict(tpch22.QUERIES)["Q22"]
    d = sess.sql(q)
    specs = [x.spec for x in d.druid_queries()]
    # the outer scan(s) + the avg(c_acctbal) subquery, all on the engine
    assert len(specs) >= 2 and any(s.queryType == "timeseries" for s in specs)
    assert any('"deferred"' in s.to_json_str(None) for s in specs)


@pytest.mark.parametrize("pattern", ["%green%", "forest%", "%rose", "%special%requests%", "%en%re%",
                                     "a%e", "%re%re%re%", "ro%ro%", "%", "%s", "g%n%e%", "%Customer%Complaints%"])
def test_words_dictionary_like(pattern):
    import re

    d = WordsDictionary(tpch.P_NAME_WORDS[:20] + ["special", "requests", "Customer", "Complaints"], 4, 5000)
    vals = d.values
    assert all(vals[i] < vals[i + 1] for i in range(len(vals) - 1))
    rx = re.compile("^" + "".join(".*" if c == "%" else re.escape(c) for c in pattern) + "$", re.S)
    exp = np.array([rx.match(v) is not None for v in vals])
    assert (d.like_mask(pattern) == exp).all()
    assert d.lookup(vals[1234]) == 1234


def test_functional_dependency_key_elimination(ds_small):
    """Q10-style wide grouping: the customer attributes are determined by o_custkey, so only the
    determinant is packed into the device key; attributes are decoded through FD tables."""
    from spark_druid_olap_amd.engine.lower import Lowerer, fd_table
    from spark_druid_olap_amd.query import spec as S

    dims = [S.DefaultDimensionSpec(d) for d in ("o_custkey", "c_name", "c_phone", "c_nation", "l_shipmode")]
    prog = Lowerer(ds_small).lower_aggregate(["1992-01-01/1999-01-01"], None, dims, None,
                                             [S.FunctionAggregationSpec("count", "n")])
    assert sorted(kc.name for kc in prog.keys) == ["l_shipmode", "o_custkey"]
    assert sorted(kc.name for kc, _, _ in prog.derived) == ["c_name", "c_nation", "c_phone"]
    assert prog.key_order == ["o_custkey", "c_name", "c_phone", "c_nation", "l_shipmode"]
    assert fd_table(ds_small, "l_shipmode", "l_returnflag") is None
    r = Engine(use_native=False).execute(S.GroupByQuerySpec("tpch", dims, aggregations=[
        S.FunctionAggregationSpec("count", "n")], intervals=["1992-01-01/1999-01-01"]), ds_small)
    assert r.columns[:5] == ["o_custkey", "c_name", "c_phone", "c_nation", "l_shipmode"]
    assert int(np.asarray(r.data["n"]).sum()) == ds_small.num_rows
    name_of = {}
    for ck, cn in zip(r.data["o_custkey"], r.data["c_name"]):
        assert name_of.setdefault(ck, cn) == cn
    assert all(str(cn).startswith("Customer#") and int(str(cn)[9:]) == int(ck)
               for ck, cn in zip(r.data["o_custkey"], r.data["c_name"]))


def test_nested_groupby_three_levels(ds_small, df_small):
    """Query data source nesting on the engine: orders per customer, then customers per order
    count (TPC-H Q13's shape) -- equal to pandas over the base rows; JSON round trip keeps it."""
    import json

    from spark_druid_olap_amd.query import spec as S

    iv = ["1992-01-01/1999-01-01"]
    inner = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("o_custkey"), S.DefaultDimensionSpec("o_orderkey")],
                               aggregations=[S.FunctionAggregationSpec("longSum", "q", "l_quantity")], intervals=iv)
    mid = S.GroupByQuerySpec(S.QueryDataSourceSpec(inner), [S.DefaultDimensionSpec("o_custkey")],
                             aggregations=[S.FunctionAggregationSpec("count", "c_count"),
                                           S.FunctionAggregationSpec("longSum", "qq", "q")], intervals=iv)
    outer = S.GroupByQuerySpec(S.QueryDataSourceSpec(mid), [S.DefaultDimensionSpec("c_count")],
                               aggregations=[S.FunctionAggregationSpec("count", "custdist"),
                                             S.FunctionAggregationSpec("longMax", "mq", "qq")], intervals=iv)
    outer = S.from_json(json.dumps(outer.to_json()))
    r = Engine(use_native=False).execute(outer, ds_small)
    got = sorted(zip(r.data["c_count"].tolist(), r.data["custdist"].tolist(), r.data["mq"].tolist()))
    g = df_small.groupby("o_custkey").agg(c=("o_orderkey", "nunique"), q=("l_quantity", "sum")).reset_index()
    e = g.groupby("c").agg(n=("o_custkey", "size"), mq=("q", "max")).reset_index()
    assert got == sorted(zip(e.c.tolist(), e.n.tolist(), [int(x) for x in e.mq.tolist()]))


@pytest.mark.parametrize("name", ["Q4", "Q13", "Q16"])
def test_two_level_aggregates_become_one_nested_query(sess, name):
    from spark_druid_olap_amd.query import spec as S

    d = sess.sql(dict(tpch22.QUERIES)[name])
    dq = d.druid_queries()
    assert len(dq) == 1 and isinstance(dq[0].spec.dataSource, S.QueryDataSourceSpec), d.explain()


def test_having_pushed_to_groupby(sess):
    d = sess.sql(dict(tpch22.QUERIES)["Q18"])
    (dq,) = d.druid_queries()
    h = dq.spec.having
    assert h is not None and h.aggregation and h.type == "greaterThan" and h.value == 300.0


def test_presence_slot_folds_into_positive_sum(ds_small, df_small):
    """sum(l_quantity) (all values >= 1) doubles as the group-presence slot: one accumulator."""
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.query import spec as S

    dims = [S.DefaultDimensionSpec("l_shipmode")]
    aggs = [S.FunctionAggregationSpec("longSum", "q", "l_quantity"),
            S.FunctionAggregationSpec("doubleSum", "e", "l_extendedprice")]
    prog = Lowerer(ds_small).lower_aggregate(["1992-01-01/1999-01-01"], None, dims, None, aggs)
    assert prog.nslots == 2 and {a.name: a.slot for a in prog.aggs}["q"] == 0
    r = Engine(use_native=False).execute(S.GroupByQuerySpec("tpch", dims, aggregations=aggs,
                                                            intervals=["1992-01-01/1999-01-01"]), ds_small)
    exp = df_small.groupby("l_shipmode")["l_quantity"].sum()
    got = dict(zip(r.data["l_shipmode"].tolist() if hasattr(r.data["l_shipmode"], "tolist") else
                   list(r.data["l_shipmode"]), r.data["q"].tolist()))
    assert {str(k): int(v) for k, v in got.items()} == {k: int(v) for k, v in exp.items()}


def test_dependent_metric_aggregate_needs_no_accumulator(ds_small, df_small):
    """max(o_totalprice) per order is read from an FD table (the metric is constant per order);
    sum(l_quantity) doubles as the presence slot: one accumulator for Q18's inner scan."""
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.query import spec as S

    dims = [S.DefaultDimensionSpec("o_orderkey")]
    aggs = [S.FunctionAggregationSpec("doubleMax", "tp", "o_totalprice"),
            S.FunctionAggregationSpec("longSum", "q", "l_quantity")]
    iv = ["1992-01-01/1999-01-01"]
    prog = Lowerer(ds_small).lower_aggregate(iv, None, dims, None, aggs)
    assert prog.nslots == 1 and [a.name for a, _, _ in prog.derived_aggs] == ["tp"]
    r = Engine(use_native=False).execute(S.GroupByQuerySpec("tpch", dims, aggregations=aggs, intervals=iv), ds_small)
    got = dict(zip(np.asarray(r.data["o_orderkey"]).tolist(), np.asarray(r.data["tp"]).tolist()))
    exp = df_small.groupby("o_orderkey")["o_totalprice"].max()
    assert len(got) == len(exp)
    for k, v in exp.items():
        assert got[int(k)] == pytest.approx(v, abs=0.005)


@pytest.mark.parametrize("q", [
    f"select c_name, o_orderkey, sum(l_quantity) from {T} where o_orderkey in "
    f"(select o_orderkey from {T} group by o_orderkey having sum(l_quantity) > 250) group by c_name, o_orderkey",
    f"select l_shipmode, count(*) from {T} where s_nation not in "
    f"(select s_nation from {T} where s_region = 'ASIA' group by s_nation) group by l_shipmode",
    f"select count(*) from {T} where p_brand in (select p_brand from {T} where p_size = 1000 group by p_brand)",
])
def test_in_subquery_pushed_as_semi_join(sess, q):
    """IN (subquery) filters run the subquery on the engine first and push the value set."""
    d = sess.sql(q)
    assert len(d.druid_queries()) == 2, d.explain()
    assert '"deferred"' in d.druid_queries()[0].spec.to_json_str(None)
    assert _rows(d) == _rows(sess.sql(q.replace(T, B)))


GLOBAL_OVER_GROUPBY = [
    # TPC-H Q15's scalar subquery shape: one device reduction over the inner groups
    f"select max(s), min(s), sum(s), count(*) from (select l_suppkey, s_name, sum(l_extendedprice) s from {T} "
    f"where l_shipdate >= '1996-01-01' and l_shipdate < '1996-04-01' group by l_suppkey, s_name) t",
    f"select count(*), max(n) from (select o_orderkey, count(*) n from {T} group by o_orderkey) t",
    # empty inner result: SQL still answers one row (count 0, the rest NULL)
    f"select count(*), max(s), sum(q) from (select s_nation, sum(l_extendedprice) s, sum(l_quantity) q from {T} "
    f"where s_nation = 'NO SUCH NATION' group by s_nation) t",
]


@pytest.mark.parametrize("i", range(len(GLOBAL_OVER_GROUPBY)))
def test_global_aggregate_over_groupby_is_nested(sess, i):
    q = GLOBAL_OVER_GROUPBY[i]
    d = sess.sql(q)
    dqs = d.druid_queries()
    assert len(dqs) == 1 and dqs[0].info.get("nested") and "global_counts" in dqs[0].info, d.explain()
    got, exp = _rows(d), _rows(sess.sql(q.replace(T, B)))
    assert len(got) == len(exp) == 1
    for a, c in zip(got[0], exp[0]):
        if isinstance(a, float) or isinstance(c, float):
            assert a == pytest.approx(c, rel=1e-9, abs=0.02), (got, exp)
        else:
            assert a == c, (got, exp)


def test_q15_subquery_runs_nested(sess):
    d = sess.sql(dict(tpch22.QUERIES)["Q15"])
    assert any(q.info.get("nested") and "global_counts" in q.info for q in d.druid_queries())


def test_deferred_scalar_subquery_sums_exactly_and_reuses_its_plan(sess):
    """A scalar subquery whose value parameterises a pushed filter runs its own pushed queries with
    exact (fixed-point) float sums: the resolved outer query is cached per value, and a float sum's
    last bits follow the device's atomic order -- every run re-planned the outer query."""
    from spark_druid_olap_amd.query.spec import find_deferred
    from spark_druid_olap_amd.sql import plan as P
    from spark_druid_olap_amd.utils import metrics as M

    q = (f"select sum(l_extendedprice) / 7.0 as avg_yearly from {T} where c_nation = 'JAPAN' and "
         f"l_quantity < (select 0.2 * avg(l_extendedprice) from {T} where c_nation = 'JAPAN')")
    d = sess.sql(q)
    first = _rows(d)
    outer = [dq for dq in d.druid_queries() if find_deferred(dq.spec)]
    assert outer, d.explain()
    inner = [dq for dq in P.find_all_deep(d.plan, P.DruidQuery) if dq not in outer]
    assert inner and all(dq.info.get("deterministic") for dq in inner)
    assert all(getattr(dq, "_prepared", None) is None or dq._prepared.deterministic for dq in inner)
    before = M.events().get("plan_prepare", 0)
    for _ in range(3):
        assert _rows(sess.sql(q)) == first
    assert M.events().get("plan_prepare", 0) == before
    # a server prepares a statement's known pushed queries before running it: the subquery's are
    # prepared exact from the start (not re-prepared when the run marks them)
    q2 = q.replace("'JAPAN'", "'CHINA'")
    d2 = sess.sql(q2)
    r0 = M.events().get("plan_reprepare", 0)
    d2.prepare()
    _rows(d2)
    assert M.events().get("plan_reprepare", 0) == r0
    assert len(outer[0].__dict__["_resolved"]) == 1
