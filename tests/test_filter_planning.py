"""The reference's FilterPlanningTest (``tsd/test/FilterPlanningTest.scala:25-157``): each WHERE
predicate must be translated into the Druid query -- an IN over dictionary values, time-column
comparisons folded into the query interval, date-string comparisons as bound filters, and the
expression predicates the reference sends as JavaScript filters (evaluated here once per dictionary
entry) -- and the pushed query must return what the same SQL returns over the base table.  The
reference asserts the exact JSON of its JavaScript filters; the equivalent check here is that
nothing is left for a host-side Filter and that the answers match."""
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.sql import plan as P

T = "orderLineItemPartSupplier"
B = "orderLineItemPartSupplierBase"

CASES = {
    "in": ("c_mktsegment in ('MACHINERY', 'HOUSEHOLD')", None),
    # 42-48: the time column compared as a timestamp -> the interval starts at 1995-12-30
    "timestamp1": ("Cast(l_shipdate AS timestamp) >= Cast('1995-12-30' AS timestamp)", ("1995-12-30", None)),
    # 50-60: to_date / concat / cast on the time column folds into the interval's end (the
    # reference ends at 1997-08-02T00:00:00.001; on a day-granular index that is the whole day)
    "timestamp2": ("Cast(Concat(To_date(l_shipdate), ' 00:00:00') AS TIMESTAMP) <= "
                   "Cast('1997-08-02 00:00:00' AS TIMESTAMP)", (None, "1997-08-03")),
    # 62-65: a string comparison on the time column (the reference keeps it in Spark; ISO date
    # strings order like dates, so it becomes an interval here)
    "timestamp3": ("l_shipdate >= '1995-12-30'", None),
    "timestamp4": ("o_orderdate >= '1995-12-30'", None),
    "timestamp5": ("Cast(Concat(To_date(o_orderdate), ' 00:00:00') AS TIMESTAMP) <= "
                   "Cast('1997-08-02 00:00:00' AS TIMESTAMP)", None),
    "monthTimestampFilter": ("Month(Cast(Concat(To_date(l_shipdate), ' 00:00:00') AS TIMESTAMP)) < 4", None),
    "jsUpper": ("upper(s_name) = 'S1'", None),
    "jsCoalesce": ("coalesce(s_name, 'no-supp') = 'S1'", None),
}


@pytest.fixture(scope="module")
def sess(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table(B, df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s


def _rows(d):
    return sorted(tuple(round(v, 2) if isinstance(v, float) else v for v in r) for r in d.collect())


@pytest.mark.parametrize("name", list(CASES))
def test_filter_is_pushed_and_exact(sess, name):
    pred, interval = CASES[name]
    sql = f"select l_returnflag, count(*), sum(l_extendedprice) from {{}} where {pred} group by l_returnflag"
    d = sess.sql(sql.format(T))
    dq = d.druid_queries()
    assert len(dq) == 1, d.explain()
    assert not any(isinstance(n, P.Filter) for n in d.plan.walk()), d.explain()  # nothing left on the host
    if interval is not None:
        ivs = dq[0].spec.to_json()["intervals"]
        lo, hi = ivs[0].split("/")
        if interval[0]:
            assert lo.startswith(interval[0]), ivs
        if interval[1]:
            assert hi.startswith(interval[1]), ivs
    got, exp = _rows(d), _rows(sess.sql(sql.format(B)))
    assert got == exp
