"""The reference's BI concurrency workload (``docs/bi-benchmark/snap-sales-demo.jmx``).

The JMeter plan drives the Thrift server with four thread groups -- "Workbook A - Low
Cardinality" (5 threads), "B - Heavy Queries" (3), "C - No Partition Filter" (2) and "D - RunOnce"
(1), each looping 5 times (``snap-sales-demo.jmx:87-101``) over its JDBC samplers in random order
(RandomOrderController) with Gaussian think times.  The sampler texts are vendored verbatim in
``templates.json``; their ``${var}`` parameters come from four CSV data sets (``:30-72``), vendored
here as ``tpchparams*.csv``:

=====================  ==============================  =====================================
CSV data set           file                            variables
=====================  ==============================  =====================================
tpchQueryParamsDate    tpchparams.csv (10 rows)        startdate, enddate
tpchQueryParamsPart.   tpchparams-pyear.csv (5 rows)   ccode1..ccode5
tpchQueryParamsPart.   tpchparams-p.csv (25 rows)      ccode1..ccode4, nation
tpchQueryParamsMkt.    tpchparams-mkt.csv (5 rows)     mktsegment
=====================  ==============================  =====================================

Every data set is ``shareMode.all`` + ``recycle``: one cursor per file shared by all threads, each
thread iteration reads the next line of every file, in plan order -- so the second
"tpchQueryParamsPartitions" set (nation names) overwrites ``ccode1..ccode4`` read from the first
(years).  ``bind="jmeter"`` reproduces that exactly (the ``p_year = "${ccodeN}"`` filters of 11
templates then compare a year with a nation name and select nothing); ``bind="years"`` keeps the
years (what the plan evidently meant).  Values are stripped of surrounding blanks (Spark's cast
to timestamp trims them too).

The templates query ``sales_demo_source`` (``docs/bi-benchmark/ec2-ddl.sql:1-42``): the flattened
TPC-H columns plus the partition columns ``p_year`` / ``p_month``, whose derivation the DDL does not
state; here they are the year / month of ``l_shipdate`` (the index timestamp), exposed as a view
over the Druid table so filters on them are pushed as single-dimension expression filters.
"""
from __future__ import annotations

import csv
import json
import os
import random
import re
from typing import Dict, Iterator, List, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))

# (file, variable names) in the plan's order (snap-sales-demo.jmx:30-72)
CSV_SETS = [("tpchparams.csv", ["startdate", "enddate"]),
            ("tpchparams-pyear.csv", ["ccode1", "ccode2", "ccode3", "ccode4", "ccode5"]),
            ("tpchparams-p.csv", ["ccode1", "ccode2", "ccode3", "ccode4", "nation"]),
            ("tpchparams-mkt.csv", ["mktsegment"])]

# thread groups (snap-sales-demo.jmx:87-101 and the later ThreadGroup elements): threads, loops
THREAD_GROUPS = {"Workbook A - Low Cardinality": (5, 5), "Workbook B - Heavy Queries": (3, 5),
                 "Workbook C - No Partition Filter": (2, 5), "Workbook D - RunOnce": (1, 5)}

# the view the templates query: the flattened table's columns named in ec2-ddl.sql:1-40 plus the
# partition columns
SOURCE_COLUMNS = ["o_orderkey", "o_orderstatus", "o_totalprice", "o_orderdate", "o_orderpriority", "o_shippriority",
                  "l_linenumber", "l_quantity", "l_extendedprice", "l_discount", "l_tax", "l_returnflag",
                  "l_linestatus", "l_shipdate", "l_commitdate", "l_receiptdate", "l_shipmode", "order_year",
                  "ps_availqty", "ps_supplycost", "s_name", "s_acctbal", "s_nation", "s_region", "p_name", "p_mfgr",
                  "p_brand", "p_type", "p_size", "p_container", "p_retailprice", "c_name", "c_phone", "c_acctbal",
                  "c_mktsegment", "c_nation", "c_region"]


def templates() -> List[Dict[str, str]]:
    """[{name, thread_group, sql}] -- the 23 enabled JDBC samplers, verbatim."""
    with open(os.path.join(HERE, "templates.json")) as f:
        return json.load(f)["templates"]


def _rows(fname: str) -> List[List[str]]:
    with open(os.path.join(HERE, fname), newline="") as f:
        return [[c.strip() for c in r] for r in csv.reader(f) if r and any(c.strip() for c in r)]


def csv_rows() -> Dict[str, List[List[str]]]:
    return {f: _rows(f) for f, _ in CSV_SETS}


def binding(k: int, bind: str = "jmeter") -> Dict[str, str]:
    """Variables of the k-th iteration (every shared cursor advanced k times)."""
    rows = csv_rows()
    out: Dict[str, str] = {}
    for fname, names in CSV_SETS:
        if bind == "years" and fname == "tpchparams-p.csv":
            names = [n if not n.startswith("ccode") else None for n in names]
        r = rows[fname][k % len(rows[fname])]
        for n, v in zip(names, r):
            if n is not None:
                out[n] = v
    return out


_VAR = re.compile(r"\$\{(\w+)\}")


def render(sql: str, vars_: Dict[str, str]) -> str:
    def sub(m):
        if m.group(1) not in vars_:
            raise KeyError(f"unbound JMeter variable ${{{m.group(1)}}}")
        return vars_[m.group(1)]
    return " ".join(_VAR.sub(sub, sql).split())


def iterations(n: int, bind: str = "jmeter") -> List[Dict[str, str]]:
    return [binding(k, bind) for k in range(n)]


def statements(n_iter: int = 25, bind: str = "jmeter") -> List[Tuple[str, str, str]]:
    """(template name, thread group, SQL) of every template under the first ``n_iter`` bindings
    (25 covers every row of every CSV file), distinct texts only."""
    out, seen = [], set()
    ts = templates()
    for k in range(n_iter):
        b = binding(k, bind)
        for t in ts:
            q = render(t["sql"], b)
            if q not in seen:
                seen.add(q)
                out.append((t["name"], t["thread_group"], q))
    return out


def client_schedule(client: int, nclients: int, bind: str = "jmeter", seed: int = 11) -> Iterator[Tuple[str, str]]:
    """The statement stream of one closed-loop client: clients are split over the thread groups in
    the plan's 5:3:2:1 proportion; each iteration takes the next binding (the shared cursors: client
    c of N starts at iteration c and steps by N) and runs its group's templates in random order."""
    groups = list(THREAD_GROUPS)
    weights = [THREAD_GROUPS[g][0] for g in groups]
    total = sum(weights)
    slots = []
    for g, w in zip(groups, weights):
        slots += [g] * max(1, round(w * nclients / total))
    group = slots[client % len(slots)]
    ts = [t for t in templates() if t["thread_group"].strip() == group]
    rnd = random.Random(seed * 1000003 + client)
    k = client
    while True:
        b = binding(k, bind)
        order = list(range(len(ts)))
        rnd.shuffle(order)
        for i in order:
            yield ts[i]["name"], render(ts[i]["sql"], b)
        k += nclients


def register(session, druid_table: str = "orderLineItemPartSupplier", name: str = "sales_demo_source") -> None:
    """``sales_demo_source`` as a view over the Druid table (see the module docstring)."""
    session.sql(view_sql(druid_table, name))


def view_sql(druid_table: str = "orderLineItemPartSupplier", name: str = "sales_demo_source") -> str:
    """A (shared-catalog) view, so every HiveServer2 client session sees it."""
    cols = ", ".join(SOURCE_COLUMNS)
    return (f"CREATE OR REPLACE VIEW {name} AS SELECT {cols}, substr(l_shipdate, 1, 4) AS p_year, "
            f"substr(l_shipdate, 6, 2) AS p_month FROM {druid_table}")
