"""The reference's DataSourceTest (``tc/DataSourceTest.scala:32-111``): the base table and the
Druid-backed table answer ``select *``, a CREATE TEMPORARY TABLE carrying a pre-built Druid query
in its ``druidQuery`` option (``sd/DefaultSource.scala:246``; the reference parses the option but
plans every scan itself, and so does this DDL), a QuerySpec run directly against a relation
(``PlanUtil.dataFrame`` -> ``ON DRUIDDATASOURCE ... EXECUTE QUERY``), and the JSON form of a
functional dependency."""
import json

import pytest

from spark_druid_olap_amd.catalog.functional_deps import FunctionalDependency
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
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


def test_base_table(sess):
    rows = sess.sql(f"select * from {B} limit 10").collect()
    assert len(rows) == 10 and len(rows[0]) == len(tpch.FLAT_SCHEMA)


def test_no_query(sess):
    d = sess.sql(f"select * from {T} limit 10")
    assert d.explain()
    assert len(d.collect()) == 10


@pytest.mark.parametrize("name", ["TPCH Q1", "Ship Date Range"])
def test_ddl_with_druid_query_option(sess, name):
    dq = json.dumps(DRUID_JSON[name]).replace("'", "")
    tmp = "orderLineItemPartSupplier2"
    sess.sql(tpch.druid_ddl(table=tmp, with_column_mapping=False,
                            star_schema=f'{{"factTable" : "{tmp}", "relations" : []}}',
                            extra_options=f", druidQuery '{dq}'").replace("CREATE TABLE if not exists",
                                                                         "CREATE TEMPORARY TABLE"))
    try:
        a = sess.sql(f"select l_returnflag, count(*) from {tmp} group by l_returnflag").collect()
        b = sess.sql(f"select l_returnflag, count(*) from {T} group by l_returnflag").collect()
        assert sorted(a) == sorted(b)
        assert len(sess.sql(f"select * from {tmp} limit 10").collect()) == 10
    finally:
        sess.sql(f"drop table if exists {tmp}")


def test_direct_query_on_relation(sess):
    # PlanUtil.dataFrame(druidRelationInfo, DruidQuery): a QuerySpec over the relation's index
    js = json.dumps(DRUID_JSON["TPCH Q1"])
    rows = sess.sql(f"on druiddatasource {T} execute query {js}").collect()
    assert rows and all(len(r) >= 3 for r in rows)


def test_functional_dependency_json():
    fd = FunctionalDependency.parse_list('[{"col1": "a", "col2": "b", "type": "1-1"}]')[0]
    assert (fd.col1, fd.col2, fd.type) == ("a", "b", "1-1")
