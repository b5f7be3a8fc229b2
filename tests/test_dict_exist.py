"""Existence-only group-bys answered over the key's dictionary domain (engine/dict_exist.py) must
return exactly the groups the row scan finds; programs whose filters read rows stay on the scan."""
import pytest

from spark_druid_olap_amd.engine import dict_exist
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.engine.lower import Lowerer
from spark_druid_olap_amd.models import tpch, tpch22
from spark_druid_olap_amd.ops.reference import run_reference
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.session import Session

ALL = ["1992-01-01T00:00:00.000Z/1999-01-01T00:00:00.000Z"]


def _sel(dim, v):
    return S.SelectorFilterSpec(dim, v)


def _prog(ds, dims, filt, intervals=None):
    low = Lowerer(ds)
    q = S.GroupByQuerySpec(ds.name, [S.DefaultDimensionSpec(d, d) for d in dims], None, None,
                           S.Granularity.parse("all"), filt, [], None, intervals or ALL)
    return low.lower_aggregate(q.intervals, q.filter, q.dimensions, q.granularity, q.aggregations)


def _keys(part):
    if part.kind == "dense":
        part = part.compact()
    return sorted(part.keys.tolist())


@pytest.mark.parametrize("case", ["comment_not_like", "customer_segment", "or_not", "key_filter"])
def test_dictionary_existence_matches_scan(ds_small, case):
    filt = {
        "comment_not_like": S.NotFilterSpec(S.RegexFilterSpec("o_comment", ".*special.*requests.*")),
        "customer_segment": _sel("c_mktsegment", "BUILDING"),
        "or_not": S.LogicalFilterSpec("or", [_sel("o_orderpriority", "1-URGENT"),
                                             S.NotFilterSpec(_sel("c_mktsegment", "MACHINERY"))]),
        "key_filter": S.BoundFilterSpec("o_orderkey", "100", "900", False, False, True),
    }[case]
    prog = _prog(ds_small, ["o_orderkey"], filt)
    pl = dict_exist.plan(prog)
    assert pl is not None and pl[0] == "o_orderkey"
    got = dict_exist.run(prog, *pl)
    assert got is not None
    exp = _keys(run_reference(prog))
    assert 0 < len(exp) < len(ds_small.dims["o_orderkey"].dictionary)  # the filter selects
    assert _keys(got) == exp


def test_row_reading_filters_stay_on_the_scan(ds_small):
    # a time restriction and a metric filter both need the rows
    p1 = _prog(ds_small, ["o_orderkey"], None, ["1994-01-01T00:00:00.000Z/1995-01-01T00:00:00.000Z"])
    assert dict_exist.plan(p1) is None
    # a line-level dimension is not determined by the order key: the rows decide
    p2 = _prog(ds_small, ["o_orderkey"], _sel("l_shipmode", "MAIL"))
    pl = dict_exist.plan(p2)
    assert pl == ("o_orderkey", ("l_shipmode",)) and dict_exist.run(p2, *pl) is None
    # two keys without an FD compaction / with aggregations: not existence-only on one dimension
    p3 = _prog(ds_small, ["l_shipmode", "l_returnflag"], None)
    assert dict_exist.plan(p3) is None


def test_q13_through_sql_uses_dictionary_domain(ds_small, df_small, monkeypatch):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    calls = []
    orig = dict_exist.run
    monkeypatch.setattr(dict_exist, "run", lambda *a, **k: calls.append(1) or orig(*a, **k))
    q = dict(tpch22.QUERIES)["Q13"]
    got = sorted(s.sql(q).collect())
    exp = sorted(s.sql(q.replace("orderLineItemPartSupplier", "orderLineItemPartSupplierBase")).collect())
    assert calls and got == exp
