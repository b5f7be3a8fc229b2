"""Filter IR rewrites in the lowering (engine/lower.py)."""
import numpy as np

from spark_druid_olap_amd.engine import lower as L


def _ids(dim, n, on):
    m = np.zeros(n, dtype=bool)
    m[list(on)] = True
    return ("ids", dim, m)


def test_or_implies_per_dimension_id_sets():
    """(a=1 & b in {0,1} & x) | (a=2 & b in {0,1} & y) == a in {1,2} & b in {0,1} & (a=1 & x | a=2 & y)."""
    x, y = ("cmp", "q", "<", 5), ("cmp", "q", ">", 9)
    e = ("or", [("and", [_ids("a", 4, [1]), _ids("b", 3, [0, 1]), x]),
                ("and", [_ids("a", 4, [2]), _ids("b", 3, [0, 1]), y])])
    out = L.imply_or_conjuncts(e)
    assert out[0] == "and"
    leaves = {c[1]: c[2] for c in out[1] if c[0] == "ids"}
    assert leaves["a"].tolist() == [False, True, True, False] and leaves["b"].tolist() == [True, True, False]
    ors = [c for c in out[1] if c[0] == "or"]
    assert len(ors) == 1
    # b's set equals the implied one in every disjunct: dropped from the OR; a's stays
    for d in ors[0][1]:
        assert all(c[1] != "b" for c in d[1] if c[0] == "ids") and any(c[1] == "a" for c in d[1] if c[0] == "ids")


def test_or_without_a_common_dimension_is_unchanged():
    e = ("or", [("and", [_ids("a", 4, [1]), ("cmp", "q", "<", 5)]), _ids("b", 3, [0])])
    assert L.imply_or_conjuncts(e) is e


def test_dimension_only_or_is_left_to_the_bitmap_prefilter():
    """(TPC-H Q7's nation pairs: the OR is bitmap-only as written; implied sets would only add leaves)"""
    e = ("or", [("and", [_ids("a", 4, [1]), _ids("b", 4, [2])]), ("and", [_ids("a", 4, [2]), _ids("b", 4, [1])])])
    assert L.imply_or_conjuncts(e) is e


def test_q19_gets_a_bitmap_prefilter_and_the_same_answer(ds_small):
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch, tpch22
    from spark_druid_olap_amd.session import Session

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    q = dict(tpch22.QUERIES)["Q19"]
    out = {}
    for flag in (True, False):
        old = L.IMPLY_OR
        L.IMPLY_OR = flag
        try:
            s._plan_cache.clear()
            df = s.sql(q)
            prog = s.engine.prepare(df.druid_query_specs()[0], ds_small).scans[0][1]
            out[flag] = (prog.pre_len, str(df.to_pandas().iloc[0, 0]))
        finally:
            L.IMPLY_OR = old
    assert out[True][0] > 0 and out[False][0] == 0
    assert out[True][1] == out[False][1]
