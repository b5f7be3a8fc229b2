"""The 8 TPC-H benchmark queries as Druid QuerySpecs (what the SQL rewrite produces for
``models/tpch.BENCH_QUERIES``; the reference publishes its planner's output for the same SQL in
``docs/benchmark/druid/queries/*.json``).  Used by GPU kernel tests on the box (where the
reference checkout is not mounted) and as a planner-independent benchmark mode."""
from __future__ import annotations

from typing import Dict, List, Tuple

from ..query import spec as S

ALL = ["1992-01-01T00:00:00.000Z/1999-01-01T00:00:00.000Z"]


def _q1_aggs():
    return [S.FunctionAggregationSpec("count", "alias-1", "count"),
            S.FunctionAggregationSpec("doubleSum", "alias-2", "l_extendedprice"),
            S.FunctionAggregationSpec("doubleMax", "alias-3", "ps_supplycost"),
            S.FunctionAggregationSpec("longSum", "alias-5", "ps_availqty"),
            S.FunctionAggregationSpec("count", "alias-6", "count"),
            S.CardinalityAggregationSpec("alias-7", ["o_orderkey"], True)]


def _avg_post():
    return [S.ArithmeticPostAggregationSpec("/", [S.FieldAccessPostAggregationSpec("alias-5"),
                                                  S.FieldAccessPostAggregationSpec("alias-6")], "alias-4")]


def _sel(d, v):
    return S.SelectorFilterSpec(d, v)


def _and(*fs):
    return S.LogicalFilterSpec("and", list(fs))


def _or(*fs):
    return S.LogicalFilterSpec("or", list(fs))


def _nation_pair():
    return _or(_and(_sel("s_nation", "FRANCE"), _sel("c_nation", "GERMANY")),
               _and(_sel("c_nation", "FRANCE"), _sel("s_nation", "GERMANY")))


def _dims(*names):
    return [S.DefaultDimensionSpec(n[0], n[1]) if isinstance(n, tuple) else S.DefaultDimensionSpec(n) for n in names]


SHIP_RANGE = ["1995-12-02T00:00:00.000Z/1997-09-03T00:00:00.000Z"]  # (1995-12-01, 1997-12-01 - 90 days]


def bench_specs() -> List[Tuple[str, S.QuerySpec]]:
    return [
        ("Basic Aggregation", S.GroupByQuerySpec("tpch", _dims("l_returnflag", "l_linestatus"),
                                                 aggregations=_q1_aggs(), postAggregations=_avg_post(),
                                                 intervals=ALL)),
        ("Ship Date Range", S.GroupByQuerySpec("tpch", _dims(("l_returnflag", "f"), ("l_linestatus", "s")),
                                               aggregations=[S.FunctionAggregationSpec("count", "alias-1", "count")],
                                               intervals=SHIP_RANGE)),
        ("SubQuery + nation,Type predicates + ShipDate Range",
         S.GroupByQuerySpec("tpch", _dims("s_nation"),
                            filter=_and(_sel("p_type", "ECONOMY ANODIZED STEEL"), _nation_pair()),
                            aggregations=_q1_aggs(), postAggregations=_avg_post(), intervals=SHIP_RANGE)),
        ("TPCH Q1", S.GroupByQuerySpec("tpch", _dims("l_returnflag", "l_linestatus"), aggregations=_q1_aggs(),
                                       postAggregations=_avg_post(), intervals=ALL)),
        ("TPCH Q3", S.GroupByQuerySpec("tpch", _dims("o_orderkey", "o_orderdate", "o_shippriority"),
                                       filter=_and(_sel("c_mktsegment", "BUILDING"),
                                                   S.BoundFilterSpec("o_orderdate", None, "1995-03-15", False, True)),
                                       aggregations=[S.FunctionAggregationSpec("doubleSum", "alias-1", "l_extendedprice")],
                                       intervals=["1995-03-16T00:00:00.000Z/1999-01-01T00:00:00.000Z"])),
        ("TPCH Q5", S.GroupByQuerySpec("tpch", _dims("s_nation"),
                                       filter=_and(_sel("s_region", "ASIA"),
                                                   S.BoundFilterSpec("o_orderdate", "1994-01-01", "1995-01-01", False, True)),
                                       aggregations=[S.FunctionAggregationSpec("doubleSum", "alias-1", "l_extendedprice")],
                                       intervals=ALL)),
        ("TPCH Q7", S.GroupByQuerySpec("tpch", _dims("s_nation", "c_nation") + [
            S.ExtractionDimensionSpec("__time", "l_shipdate", S.TimeFormatExtractionFunctionSpec("yyyy"))],
            filter=_nation_pair(),
            aggregations=[S.FunctionAggregationSpec("doubleSum", "alias-1", "l_extendedprice")], intervals=ALL)),
        ("TPCH Q8", S.GroupByQuerySpec("tpch", [S.ExtractionDimensionSpec(
            "o_orderdate", "o_orderdate", S.TimeParsingExtractionFunctionSpec("yyyy-MM-dd", "yyyy"))],
            filter=_and(_sel("c_region", "AMERICA"), _sel("p_type", "ECONOMY ANODIZED STEEL"),
                        S.BoundFilterSpec("o_orderdate", "1995-01-01", "1996-12-31", False, False)),
            aggregations=[S.FunctionAggregationSpec("doubleSum", "alias-1", "l_extendedprice")], intervals=ALL)),
    ]


DRUID_JSON: Dict[str, dict] = {name: q.to_json() for name, q in bench_specs()}
