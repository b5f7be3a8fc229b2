"""Window functions (sql/window.py): ranking, offset and framed aggregate functions over plain rows
and over a pushed Druid aggregate, checked against pandas / hand-computed answers."""
import numpy as np
import pandas as pd
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session


@pytest.fixture(scope="module")
def sess():
    s = Session(engine=Engine(use_native=False))
    df = pd.DataFrame({"g": ["a", "a", "a", "b", "b", "c"], "o": [1, 2, 2, 1, 3, 5],
                       "v": [1.0, 2.0, 3.0, 4.0, None, 6.0]})
    s.register_table("t", df)
    return s


def test_ranking_and_running_frames(sess):
    r = sess.sql("select g, o, v, row_number() over (partition by g order by o) rn, "
                 "rank() over (partition by g order by o) rk, dense_rank() over (partition by g order by o) dr, "
                 "sum(v) over (partition by g order by o) rs, count(v) over (partition by g) c, "
                 "avg(v) over (partition by g) pa from t order by g, o, v").collect()
    assert [x[3] for x in r] == [1, 2, 3, 1, 2, 1]
    assert [x[4] for x in r] == [1, 2, 2, 1, 2, 1]       # peers share a rank
    assert [x[5] for x in r] == [1, 2, 2, 1, 2, 1]
    assert [x[6] for x in r] == [1.0, 6.0, 6.0, 4.0, 4.0, 6.0]  # RANGE .. CURRENT ROW includes peers
    assert [x[7] for x in r] == [3, 3, 3, 1, 1, 1]
    assert [x[8] for x in r] == [2.0, 2.0, 2.0, 4.0, 4.0, 6.0]


def test_row_frames_and_offsets(sess):
    r = sess.sql("select g, o, v, max(v) over (partition by g order by o, v rows between 1 preceding and current row) m, "
                 "sum(v) over (order by g, o, v rows between 1 preceding and 1 following) s3, "
                 "lag(v) over (partition by g order by o, v) lg, lead(o, 1, -1) over (partition by g order by o, v) ld, "
                 "first_value(v) over (partition by g order by o, v) fv from t order by g, o, v").collect()
    assert [x[3] for x in r] == [1.0, 2.0, 3.0, 4.0, 4.0, 6.0]
    vals = [1.0, 2.0, 3.0, 4.0, 0.0, 6.0]  # NULL contributes nothing to the sum
    exp = [sum(vals[max(0, i - 1):i + 2]) for i in range(6)]
    assert [x[4] for x in r] == pytest.approx(exp)
    assert [x[5] for x in r] == [None, 1.0, 2.0, None, 4.0, None]
    assert [x[6] for x in r] == [2, 2, -1, 3, -1, -1]
    assert [x[7] for x in r] == [1.0, 1.0, 1.0, 4.0, 4.0, 6.0]


def test_window_over_filtered_subquery(sess):
    r = sess.sql("select g, o from (select g, o, rank() over (partition by g order by o desc) r from t) x "
                 "where r = 1 order by g, o").collect()
    assert r == [("a", 2), ("a", 2), ("b", 3), ("c", 5)]


def test_window_over_pushed_aggregate(ds_small, df_small):
    """The BI workload's shape: the group-by is pushed to the engine, the window runs over its rows."""
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    q = ("select p_mfgr, p_brand, sum(l_extendedprice) as revenue, "
         "sum(l_extendedprice) - max(sum(l_extendedprice)) over (partition by p_mfgr order by sum(l_extendedprice) desc) "
         "as delta, dense_rank() over (partition by p_mfgr order by sum(l_extendedprice) desc) rk "
         "from orderLineItemPartSupplier group by p_mfgr, p_brand")
    d = s.sql(q)
    assert d.druid_queries()
    got = d.to_pandas()
    g = df_small.groupby(["p_mfgr", "p_brand"]).l_extendedprice.sum().reset_index(name="revenue")
    g["top"] = g.groupby("p_mfgr").revenue.transform("max")
    g["rk"] = g.groupby("p_mfgr").revenue.rank(method="dense", ascending=False).astype(int)
    m = got.merge(g, on=["p_mfgr", "p_brand"], suffixes=("", "_e"))
    assert len(m) == len(g) == len(got)
    np.testing.assert_allclose(m.revenue, m.revenue_e)
    np.testing.assert_allclose(m.delta, m.revenue_e - m.top)
    assert (m.rk == m.rk_e).all()


@pytest.mark.parametrize("fn,order,partition", [("dense_rank", "asc", "p_mfgr"), ("rank", "desc", "p_mfgr"),
                                                  ("rank", "asc", "p_mfgr, s_region"), ("dense_rank", "desc", "c_region")])
def test_rank_one_pushdown(ds_small, df_small, fn, order, partition):
    """rank() / dense_rank() = 1 over a pushed groupBy (the BI plan's MinCost template): the
    groupBy carries a device pre-filter (sql/window.py push_rank_one) and the answer equals the
    unpushed plan's and pandas'."""
    from spark_druid_olap_amd.sql import plan as P

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    keys = ["p_mfgr", "p_brand", "s_region", "c_region"]
    q = (f"select {', '.join(keys)}, cnt from (select {', '.join(keys)}, count(*) cnt, "
         f"{fn}() over (partition by {partition} order by sum(l_quantity) {order}) rk "
         f"from orderLineItemPartSupplier group by {', '.join(keys)}) t where rk = 1")
    d = s.sql(q)
    dqs = P.find_all_deep(d.plan, P.DruidQuery)
    assert dqs and dqs[0].info.get("partition_extreme") is not None
    got = sorted(d.collect())
    s.conf.set("spark.sparklinedata.druid.window.rankone.pushdown", "false")
    s._plan_cache.clear()
    d0 = s.sql(q)
    assert not P.find_all_deep(d0.plan, P.DruidQuery)[0].info.get("partition_extreme")
    assert got == sorted(d0.collect())
    g = df_small.groupby(keys).agg(cnt=("l_quantity", "size"), q=("l_quantity", "sum")).reset_index()
    parts = [x.strip() for x in partition.split(",")]
    ext = g.groupby(parts).q.transform("min" if order == "asc" else "max")
    want = sorted(tuple(r) for r in g[g.q == ext][keys + ["cnt"]].itertuples(index=False, name=None))
    assert got == want


def test_rank_safe_casts():
    from spark_druid_olap_amd.sql.window import _rank_safe_cast

    assert _rank_safe_cast("int", "bigint") and _rank_safe_cast("smallint", "int")
    assert _rank_safe_cast("bigint", "double") and _rank_safe_cast("float", "double")
    assert not _rank_safe_cast("double", "int") and not _rank_safe_cast("double", "float")
    assert not _rank_safe_cast("bigint", "int") and not _rank_safe_cast("double", "bigint")


@pytest.mark.parametrize("order_expr,pushed", [("cast(sum(l_extendedprice) as int)", False),
                                               ("cast(sum(l_extendedprice) as float)", False),
                                               ("cast(count(*) as int)", False)])
def test_rank_one_pushdown_through_casts(ds_small, df_small, order_expr, pushed):
    """The rank-one pre-filter only looks through casts that are injective for the metric's type:
    cast(sum(double) as int) maps distinct sums to one value (1.2 and 1.7 both rank 1 in Spark), so
    the device must not keep only the partition minimum of the uncast sum."""
    from spark_druid_olap_amd.sql import plan as P

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    q = ("select p_mfgr, p_brand, cnt from (select p_mfgr, p_brand, count(*) cnt, "
         f"dense_rank() over (partition by p_mfgr order by {order_expr}) rk "
         "from orderLineItemPartSupplier group by p_mfgr, p_brand) t where rk = 1")
    d = s.sql(q)
    dqs = P.find_all_deep(d.plan, P.DruidQuery)
    assert dqs and bool(dqs[0].info.get("partition_extreme")) == pushed
    got = sorted(d.collect())
    s.conf.set("spark.sparklinedata.druid.window.rankone.pushdown", "false")
    s._plan_cache.clear()
    assert got == sorted(s.sql(q).collect())


def test_window_errors(sess):
    from spark_druid_olap_amd.sql.types import AnalysisError

    with pytest.raises(AnalysisError):
        sess.sql("select g from t where rank() over (order by o) = 1")
    with pytest.raises(AnalysisError):
        sess.sql("select upper(g) over (order by o) from t")


def test_integer_frame_sums_exact():
    """Framed sums of bigint arguments stay exact above 2^53 (Spark's sum(bigint) is exact)."""
    s = Session(engine=Engine(use_native=False))
    big = 2 ** 60
    s.register_table("w", pd.DataFrame({"g": [1, 1, 1, 1], "o": [1, 2, 3, 4],
                                        "v": np.array([big, 3, 5, 7], dtype=np.int64)}))
    r = s.sql("select o, sum(v) over (partition by g order by o) rs, "
              "sum(v) over (partition by g order by o rows between 1 preceding and current row) m2 "
              "from w order by o").collect()
    assert [int(x[1]) for x in r] == [big, big + 3, big + 8, big + 15]
    assert [int(x[2]) for x in r] == [big, big + 3, 8, 12]
