"""Star-schema join elimination (the reference's JoinTransform; tc/StarSchemaTpchQueriesCTest.scala,
tc/JoinTest.scala, tc/StarSchemaMetadataTest.scala): TPC-H queries written over lineitem ⋈ orders ⋈
customer ⋈ ... collapse into ONE Druid query over the denormalized index and match the same SQL run
as real joins over the base tables."""
import re

import pytest

from spark_druid_olap_amd.catalog.star_schema import StarSchema, StarSchemaError, StarSchemaInfo
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session

Q = {
    "q1": """select l_returnflag, l_linestatus, count(*), sum(l_extendedprice) as s, max(ps_supplycost) as m,
             avg(ps_availqty) as a from lineitem, partsupp, orders
             where dateIsBeforeOrEqual(dateTime(l_shipdate), dateMinus(dateTime('1997-12-01'), period('P90D')))
               and l_orderkey = o_orderkey and l_suppkey = ps_suppkey and l_partkey = ps_partkey
             group by l_returnflag, l_linestatus""",
    "q3": """select o_orderkey, sum(l_extendedprice) as price, o_orderdate, o_shippriority
             from customer, orders, lineitem
             where c_mktsegment = 'BUILDING' and dateIsBefore(dateTime(o_orderdate), dateTime('1995-03-15'))
               and dateIsAfter(dateTime(l_shipdate), dateTime('1995-03-15'))
               and c_custkey = o_custkey and l_orderkey = o_orderkey
             group by o_orderkey, o_orderdate, o_shippriority""",
    "q5": """select sn_name, sum(l_extendedprice) as extendedPrice
             from customer, orders, lineitem, partsupp, supplier, suppnation, suppregion
             where c_custkey = o_custkey and l_orderkey = o_orderkey and l_suppkey = ps_suppkey
               and l_partkey = ps_partkey and ps_suppkey = s_suppkey and s_nationkey = sn_nationkey
               and sn_regionkey = sr_regionkey and sr_name = 'ASIA'
               and dateIsAfterOrEqual(dateTime(o_orderdate), dateTime('1994-01-01'))
               and dateIsBefore(dateTime(o_orderdate), datePlus(dateTime('1994-01-01'), period('P1Y')))
             group by sn_name""",
    "q7": """select sn_name, cn_name, year(dateTime(l_shipdate)) as l_year, sum(l_extendedprice) as ep
             from partsupp, supplier, lineitem, orders, customer, suppnation n1, custnation n2
             where ps_partkey = l_partkey and ps_suppkey = l_suppkey and ps_suppkey = s_suppkey
               and o_orderkey = l_orderkey and c_custkey = o_custkey and s_nationkey = n1.sn_nationkey
               and c_nationkey = n2.cn_nationkey
               and ((sn_name = 'FRANCE' and cn_name = 'GERMANY') or (cn_name = 'FRANCE' and sn_name = 'GERMANY'))
             group by sn_name, cn_name, year(dateTime(l_shipdate))""",
    "q8": """select year(dateTime(o_orderdate)) as o_year, sum(l_extendedprice) as price
             from partsupp, part, supplier, lineitem, orders, customer, custnation n1, suppnation n2, custregion
             where ps_partkey = l_partkey and ps_suppkey = l_suppkey and ps_partkey = p_partkey
               and ps_suppkey = s_suppkey and l_orderkey = o_orderkey and o_custkey = c_custkey
               and c_nationkey = n1.cn_nationkey and n1.cn_regionkey = cr_regionkey
               and s_nationkey = n2.sn_nationkey and cr_name = 'AMERICA' and p_type = 'ECONOMY ANODIZED STEEL'
               and dateIsAfterOrEqual(dateTime(o_orderdate), dateTime('1995-01-01'))
               and dateIsBeforeOrEqual(dateTime(o_orderdate), dateTime('1996-12-31'))
             group by year(dateTime(o_orderdate))""",
    "q10": """select c_name, cn_name, c_address, c_phone, c_comment, sum(l_extendedprice) as price
              from customer, orders, lineitem, custnation
              where c_custkey = o_custkey and l_orderkey = o_orderkey and c_nationkey = cn_nationkey
                and dateIsAfterOrEqual(dateTime(o_orderdate), dateTime('1993-10-01'))
                and dateIsBefore(dateTime(o_orderdate), datePlus(dateTime('1993-10-01'), period('P3M')))
                and l_returnflag = 'R'
              group by c_name, cn_name, c_address, c_phone, c_comment""",
}


@pytest.fixture(scope="module")
def sess(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    for name, frame in tpch.star_tables(df_small).items():
        s.register_table(name, frame, schema=tpch.STAR_SCHEMAS[name])
    # the bench-profile index keeps l_quantity / ps_availqty names: map only the nation/region renames
    s.sql(tpch.star_ddl(column_mapping=tpch.STAR_COLUMN_MAPPING))
    return s


def _norm(rows):
    return sorted([tuple(round(v, 2) if isinstance(v, float) else v for v in r) for r in rows],
                  key=lambda r: tuple((x is None, str(x)) for x in r))


@pytest.mark.parametrize("name", sorted(Q))
def test_star_query_eliminates_joins(sess, name):
    q = Q[name]
    d = sess.sql(q)
    dq = d.druid_queries()
    assert len(dq) == 1, d.explain()
    assert not any(type(p).__name__ == "Join" for p in d.plan.walk()), d.explain()
    base = sess.sql(re.sub(r"\blineitem\b", "lineitembase", q))
    assert not base.druid_queries()
    got, exp = _norm(d.collect()), _norm(base.collect())
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        for x, y in zip(a, b):
            if isinstance(x, float) or isinstance(y, float):
                assert x == pytest.approx(y, rel=1e-9, abs=0.02)
            else:
                assert x == y


def test_non_star_join_not_eliminated(sess):
    # joining lineitem to customer directly is not a declared star join (customer hangs off orders)
    d = sess.sql("select c_mktsegment, count(*) from lineitem, customer where l_orderkey = c_custkey "
                 "group by c_mktsegment")
    assert not any(len(x.spec.__dict__.get("dimensions", [])) and "c_mktsegment" in str(x.spec.to_json())
                   for x in d.druid_queries())


def test_star_schema_validation():
    cols = {"f": ["a", "b"], "d1": ["k1", "x"], "d2": ["k2", "x"]}
    ok = StarSchemaInfo.parse({"factTable": "f", "relations": [
        {"leftTable": "f", "rightTable": "d1", "relationType": "n-1",
         "joinCondition": [{"leftAttribute": "a", "rightAttribute": "k1"}]}]})
    s = StarSchema.build("f", ok, lambda t: cols[t.split(".")[-1]])
    assert s.is_star_join(["a"], ["k1"]) == ("f", "d1")
    assert s.is_star_join(["k1"], ["a"]) == ("d1", "f")
    assert s.is_star_join(["b"], ["k1"]) is None
    dup = StarSchemaInfo.parse({"factTable": "f", "relations": [
        {"leftTable": "f", "rightTable": "d1", "relationType": "n-1",
         "joinCondition": [{"leftAttribute": "a", "rightAttribute": "k1"}]},
        {"leftTable": "f", "rightTable": "d2", "relationType": "n-1",
         "joinCondition": [{"leftAttribute": "b", "rightAttribute": "k2"}]}]})
    with pytest.raises(StarSchemaError, match="not unique"):
        StarSchema.build("f", dup, lambda t: cols[t.split(".")[-1]])
    with pytest.raises(StarSchemaError, match="not part of the join Graph"):
        StarSchema.build("f", StarSchemaInfo.parse({"factTable": "f", "relations": [
            {"leftTable": "d1", "rightTable": "d2", "relationType": "n-1",
             "joinCondition": [{"leftAttribute": "k1", "rightAttribute": "k2"}]}]}),
            lambda t: {"f": ["a"], "d1": ["k1"], "d2": ["k2"]}[t.split(".")[-1]])


def test_cached_dimension_tables_still_star_join(sess):
    """CACHE TABLE on dimension tables (``spark.sparklinedata.druid.cache.tables.tocheck``, the
    reference's CachedTablePattern, ``asql/CachedTablePattern.scala:39-158``): a cached copy is
    the same catalog relation here, so the star join is still recognised and eliminated."""
    for t in ("customer", "orders"):
        sess.sql(f"CACHE TABLE {t}")
    try:
        d = sess.sql(Q["q3"])
        assert len(d.druid_queries()) == 1
        assert not any(type(p).__name__ == "Join" for p in d.plan.walk()), d.explain()
    finally:
        for t in ("customer", "orders"):
            sess.sql(f"UNCACHE TABLE {t}")


# --- the reference's StarSchemaMetadataTest (tc/StarSchemaMetadataTest.scala:27-118) ----------
def _rel(left, right, *pairs):
    return {"leftTable": left, "rightTable": right, "relationType": "n-1",
            "joinCondition": [{"leftAttribute": a, "rightAttribute": b} for a, b in pairs]}


def _build(*rels):
    def cols(t):
        t = t.split(".")[-1]
        t = {"lineitem": "lineitembase", "partsupp2": "partsupp"}.get(t, t)
        return [c for c, _ in tpch.STAR_SCHEMAS[t]]
    return StarSchema.build("lineitem", StarSchemaInfo.parse({"factTable": "lineitem", "relations": list(rels)}), cols)


_TPCH_RELS = [
    _rel("lineitem", "orders", ("l_orderkey", "o_orderkey")),
    _rel("lineitem", "partsupp", ("l_partkey", "ps_partkey"), ("l_suppkey", "ps_suppkey")),
    _rel("partsupp", "part", ("ps_partkey", "p_partkey")),
    _rel("partsupp", "supplier", ("ps_suppkey", "s_suppkey")),
    _rel("orders", "customer", ("o_custkey", "c_custkey")),
    _rel("customer", "custnation", ("c_nationkey", "cn_nationkey")),
    _rel("custnation", "custregion", ("cn_regionkey", "cr_regionkey")),
    _rel("supplier", "suppnation", ("s_nationkey", "sn_nationkey")),
    _rel("suppnation", "suppregion", ("sn_regionkey", "sr_regionkey")),
]


@pytest.mark.parametrize("rels", [
    _TPCH_RELS[:1],                                                                          # simpleStar
    [_TPCH_RELS[0], _rel("lineitem", "part", ("l_partkey", "p_partkey")),
     _rel("lineitem", "supplier", ("l_suppkey", "s_suppkey"))],                              # salesStar
    _TPCH_RELS,                                                                              # tpch
], ids=["simpleStar", "salesStar", "tpch"])
def test_valid_star_schemas(rels):
    s = _build(*rels)
    assert s.is_star_join(["l_orderkey"], ["o_orderkey"]) == ("lineitem", "orders")


def test_multiple_paths_not_allowed():
    with pytest.raises(StarSchemaError, match="multiple join paths to table 'supplier'"):
        _build(*_TPCH_RELS[:4], _rel("lineitem", "supplier", ("l_suppkey", "s_suppkey")))


def test_non_unique_columns_not_allowed():
    with pytest.raises(StarSchemaError, match="Column ps_partkey is not unique across Star Schema"):
        _build(*_TPCH_RELS[:4], _rel("lineitem", "partsupp2", ("l_partkey", "ps_partkey"), ("l_suppkey", "ps_suppkey")))
