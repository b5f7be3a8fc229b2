"""Star Schema Benchmark (SSB) model family -- BASELINE.json config 4 ("SSB SF=300 topN +
countDistinct(HLL) on dictionary-encoded dims, 8 GPU").

The reference's own index specs cover TPC-H and zip codes only; SSB is the standard star-schema
OLAP benchmark (O'Neil et al.) over ``lineorder`` + ``customer`` / ``supplier`` / ``part`` /
``dwdate``, and exercises exactly the reference's capability set: star-join elimination
(``asd/JoinTransform.scala``), dimension filters pushed as Druid filters, group-by over
dictionary-encoded dimension attributes, topN (``sd/query/QuerySpecTransforms.scala:279-332``)
and approximate count-distinct (``asd/AggregateTransform.scala:454-479``).

As with TPC-H (models/tpch.py) the data is synthetic and generated on the device: ``lineorder``
rows with dbgen-like distributions, dimension attributes derived from the keys by integer hashing
(identical on every rank, nothing materialized), the Druid index is the denormalized
``lineorder`` (time dimension ``lo_orderdate``) whose dimensions are the dimension tables'
attributes.  Weak scaling: each rank owns a contiguous ``lo_orderkey`` range.
"""
from __future__ import annotations

import json
import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..query.intervals import civil_from_days, days_from_civil
from ..segment.datasource import DataSource, make_datasource
from ..segment.dictionary import LONG, STRING, Dictionary, FormattedDictionary, RangeDictionary
from .tpch import NATIONS, REGIONS, SEGMENTS, PRIORITIES, SHIPMODES, FlatTPCH, _sorted_codes, khash

START_DAY = days_from_civil(1992, 1, 1)
END_DAY = days_from_civil(1998, 12, 31)
ORDER_SPAN = days_from_civil(1998, 8, 2) - START_DAY + 1
MONTHS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]
COLORS = ["almond", "antique", "aquamarine", "azure", "beige", "bisque", "black", "blanched", "blue", "blush",
          "brown", "burlywood", "burnished", "chartreuse", "chiffon", "chocolate", "coral", "cornflower",
          "cornsilk", "cream", "cyan", "dark", "deep", "dim", "dodger", "drab", "firebrick", "floral", "forest",
          "frosted", "gainsboro", "ghost", "goldenrod", "green", "grey", "honeydew", "hot", "indian", "ivory",
          "khaki", "lace", "lavender", "lawn", "lemon", "light", "lime", "linen", "magenta", "maroon", "medium",
          "metallic", "midnight", "mint", "misty", "moccasin", "navajo", "navy", "olive", "orange", "orchid",
          "pale", "papaya", "peach", "peru", "pink", "plum", "powder", "puff", "purple", "red", "rose", "rosy",
          "royal", "saddle", "salmon", "sandy", "seashell", "sienna", "sky", "slate", "smoke", "snow", "spring",
          "steel", "tan", "thistle", "tomato", "turquoise", "violet", "wheat", "white", "yellow"]
TYPES = [f"{a} {b} {c}" for a in ["STANDARD", "SMALL", "MEDIUM", "LARGE", "ECONOMY", "PROMO"]
         for b in ["ANODIZED", "BURNISHED", "PLATED", "POLISHED", "BRUSHED"]
         for c in ["TIN", "NICKEL", "BRASS", "STEEL", "COPPER"]]
CONTAINERS = [f"{a} {b}" for a in ["SM", "LG", "MED", "JUMBO", "WRAP"]
              for b in ["CASE", "BOX", "BAG", "JAR", "PKG", "PACK", "CAN", "DRUM"]]


def city_names() -> List[str]:
    """SSB cities: the first 9 characters of the nation name + a digit (250 values)."""
    return [f"{n[:9]:<9}{d}" for n, _ in NATIONS for d in range(10)]


def _date_attrs(d0: int, d1: int) -> Dict[str, list]:
    """dwdate rows for days d0..d1 (SSB: d_datekey yyyymmdd, d_yearmonthnum yyyymm, 'Jan1994', ...)."""
    out = {k: [] for k in ("d_datekey", "d_date", "d_dayofweek", "d_month", "d_year", "d_yearmonthnum",
                           "d_yearmonth", "d_daynuminweek", "d_daynuminmonth", "d_daynuminyear",
                           "d_monthnuminyear", "d_weeknuminyear", "d_sellingseason")}
    dows = ["Thursday", "Friday", "Saturday", "Sunday", "Monday", "Tuesday", "Wednesday"]  # 1970-01-01 = Thu
    for d in range(d0, d1 + 1):
        y, m, dd = civil_from_days(d)
        doy = d - days_from_civil(y, 1, 1) + 1
        out["d_datekey"].append(y * 10000 + m * 100 + dd)
        out["d_date"].append(f"{MONTHS[m - 1]} {dd}, {y}")
        out["d_dayofweek"].append(dows[d % 7])
        out["d_month"].append(MONTHS[m - 1])
        out["d_year"].append(y)
        out["d_yearmonthnum"].append(y * 100 + m)
        out["d_yearmonth"].append(f"{MONTHS[m - 1]}{y}")
        out["d_daynuminweek"].append((d + 3) % 7 + 1)
        out["d_daynuminmonth"].append(dd)
        out["d_daynuminyear"].append(doy)
        out["d_monthnuminyear"].append(m)
        out["d_weeknuminyear"].append((doy - 1) // 7 + 1)
        out["d_sellingseason"].append("Christmas" if m == 12 else "Summer" if m in (6, 7, 8) else
                                      "Winter" if m in (1, 2) else "Spring" if m in (3, 4, 5) else "Fall")
    return out


def sizes(sf: float, world: int = 1) -> Dict[str, int]:
    tot = sf * world
    return {"orders": max(8, int(round(1_500_000 * sf))), "customers": max(10, int(round(30_000 * tot))),
            "suppliers": max(4, int(round(2_000 * tot))),
            "parts": max(20, int(round(200_000 * (1 + math.floor(math.log2(max(tot, 1.0))))))) if tot >= 1
            else max(20, int(round(200_000 * tot)))}


def generate_flat(sf: float = 1.0, device="cpu", rank: int = 0, world: int = 1, seed: int = 19920101) -> FlatTPCH:
    """This rank's share of SSB lineorder (SF per rank), denormalized with every dimension attribute."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed * 1000 + rank)
    sz = sizes(sf, world)
    No, C, S, P = sz["orders"], sz["customers"], sz["suppliers"], sz["parts"]

    def rint(lo, hi, n, dtype=torch.int32):
        return torch.randint(lo, hi, (n,), generator=g, device=dev, dtype=dtype)

    orderkey = torch.arange(No, device=dev, dtype=torch.int64) + rank * No + 1
    odate = rint(0, ORDER_SPAN, No) + START_DAY
    custkey = rint(1, C + 1, No, torch.int64)
    opri = rint(0, 5, No, torch.int16)
    nlines = rint(1, 8, No, torch.int64)
    L = int(nlines.sum().item())
    oidx = torch.repeat_interleave(torch.arange(No, device=dev, dtype=torch.int64), nlines)
    od = odate[oidx]
    perm = torch.argsort(od, stable=True)
    oidx, od = oidx[perm], od[perm]
    del perm
    pk = rint(1, P + 1, L, torch.int64)
    sk = rint(1, S + 1, L, torch.int64)
    qty = rint(1, 51, L, torch.int64)
    disc = rint(0, 11, L, torch.int64)
    tax = rint(0, 9, L, torch.int64)
    smode = rint(0, 7, L, torch.uint8)
    price = 90000 + torch.remainder(pk // 10, 20001) + 100 * torch.remainder(pk, 1000)   # cents
    ext = qty * price
    revenue = torch.div(ext * (100 - disc), 100, rounding_mode="floor")
    supplycost = torch.div(price * 6, 10, rounding_mode="floor")
    ck = custkey[oidx]
    ototal = torch.zeros(No, dtype=torch.int64, device=dev).index_add_(0, oidx, revenue)[oidx]

    flat = FlatTPCH(sf, rank, world, L, od.to(torch.int32))
    flat.counts = {"orders": No * world, "customers": C, "parts": P, "suppliers": S}

    def dim(name, d, ids):
        flat.dims[name] = (d, ids)

    def num(name, t, kind, scale=0):
        flat.nums[name] = (t, kind, scale)

    # lineorder (numeric columns double as low-cardinality dimensions, like the reference's index
    # where l_discount / l_quantity are filterable)
    dim("lo_orderkey", RangeDictionary(1, No * world), (orderkey[oidx] - 1).to(torch.int32))
    dim("lo_custkey", RangeDictionary(1, C), (ck - 1).to(torch.int32))
    dim("lo_partkey", RangeDictionary(1, P), (pk - 1).to(torch.int32))
    dim("lo_suppkey", RangeDictionary(1, S), (sk - 1).to(torch.int32))
    dim("lo_orderpriority", Dictionary(PRIORITIES), opri[oidx].to(torch.uint8))
    dim("lo_shipmode", Dictionary(SHIPMODES), smode)
    dim("lo_quantity", Dictionary(list(range(1, 51)), LONG), (qty - 1).to(torch.uint8))
    dim("lo_discount", Dictionary(list(range(0, 11)), LONG), disc.to(torch.uint8))
    dim("lo_tax", Dictionary(list(range(0, 9)), LONG), tax.to(torch.uint8))
    num("lo_extendedprice", ext.to(torch.int32) if int(ext.max()) < 2 ** 31 else ext, "long")
    num("lo_revenue", revenue.to(torch.int32) if int(revenue.max()) < 2 ** 31 else revenue, "long")
    num("lo_supplycost", supplycost.to(torch.int32), "long")
    num("lo_ordtotalprice", ototal, "long")
    # dwdate attributes of the order date
    da = _date_attrs(START_DAY, END_DAY)
    di = (od - START_DAY).to(torch.int64)
    for col, vals, vt in (("d_year", da["d_year"], LONG), ("d_yearmonthnum", da["d_yearmonthnum"], LONG),
                          ("d_weeknuminyear", da["d_weeknuminyear"], LONG),
                          ("d_yearmonth", da["d_yearmonth"], STRING), ("d_month", da["d_month"], STRING),
                          ("d_dayofweek", da["d_dayofweek"], STRING),
                          ("d_sellingseason", da["d_sellingseason"], STRING)):
        uniq = sorted(set(vals), key=(lambda v: v))
        pos = {v: i for i, v in enumerate(uniq)}
        remap = torch.tensor([pos[v] for v in vals], dtype=torch.int64, device=dev)
        dim(col, Dictionary(uniq, vt), remap[di].to(torch.uint8))
    # customer
    cities = city_names()
    city_d, city_remap = _sorted_codes(cities)
    city_t = torch.from_numpy(city_remap).to(dev)
    nat_d, nat_remap = _sorted_codes([n for n, _ in NATIONS])
    nat_t = torch.from_numpy(nat_remap).to(dev)
    reg_of_nat = torch.tensor([r for _, r in NATIONS], device=dev, dtype=torch.int64)
    reg_d = Dictionary(REGIONS, STRING)
    c_city = khash(ck, 21) % 250
    dim("c_name", FormattedDictionary("Customer#", 9, C, start=1), (ck - 1).to(torch.int32))
    dim("c_city", city_d, city_t[c_city].to(torch.uint8))
    dim("c_nation", nat_d, nat_t[c_city // 10].to(torch.uint8))
    dim("c_region", reg_d, reg_of_nat[c_city // 10].to(torch.uint8))
    dim("c_mktsegment", Dictionary(SEGMENTS), (khash(ck, 22) % 5).to(torch.uint8))
    # supplier
    s_city = khash(sk, 31) % 250
    dim("s_name", FormattedDictionary("Supplier#", 9, S, start=1), (sk - 1).to(torch.int32))
    dim("s_city", city_d, city_t[s_city].to(torch.uint8))
    dim("s_nation", nat_d, nat_t[s_city // 10].to(torch.uint8))
    dim("s_region", reg_d, reg_of_nat[s_city // 10].to(torch.uint8))
    # part: mfgr 1..5, category mfgr*10 + 1..5, brand1 category*100 + 1..40
    mf = khash(pk, 41) % 5 + 1
    cat = mf * 10 + khash(pk, 42) % 5 + 1
    br = cat * 100 + khash(pk, 43) % 40 + 1
    dim("p_name", FormattedDictionary("part-", 9, P, start=1), (pk - 1).to(torch.int32))
    dim("p_mfgr", Dictionary([f"MFGR#{i}" for i in range(1, 6)]), (mf - 1).to(torch.uint8))
    cats = [f"MFGR#{m}{c}" for m in range(1, 6) for c in range(1, 6)]
    dim("p_category", Dictionary(cats), ((mf - 1) * 5 + (cat % 10) - 1).to(torch.uint8))
    brands = [f"MFGR#{m}{c}{b:02d}" for m in range(1, 6) for c in range(1, 6) for b in range(1, 41)]
    dim("p_brand1", Dictionary(brands), (((mf - 1) * 5 + (cat % 10) - 1) * 40 + (br % 100) - 1).to(torch.int16))
    col_d, col_remap = _sorted_codes(COLORS)
    dim("p_color", col_d, torch.from_numpy(col_remap).to(dev)[khash(pk, 44) % len(COLORS)].to(torch.uint8))
    typ_d, typ_remap = _sorted_codes(TYPES)
    dim("p_type", typ_d, torch.from_numpy(typ_remap).to(dev)[khash(pk, 45) % len(TYPES)].to(torch.uint8))
    dim("p_size", Dictionary(list(range(1, 51)), LONG), (khash(pk, 46) % 50).to(torch.uint8))
    con_d, con_remap = _sorted_codes(CONTAINERS)
    dim("p_container", con_d, torch.from_numpy(con_remap).to(dev)[khash(pk, 47) % 40].to(torch.uint8))
    return flat


INDEX_METRICS = {"lo_extendedprice": "long", "lo_revenue": "long", "lo_supplycost": "long",
                 "lo_ordtotalprice": "long"}


def to_datasource(flat: FlatTPCH, name: str = "ssb", bitmap_max_card: int = 256) -> DataSource:
    dim_ids = {k: ids for k, (_, ids) in flat.dims.items()}
    dicts = {k: d for k, (d, _) in flat.dims.items()}
    mdata = {k: t for k, (t, _, _) in flat.nums.items()}
    mkinds = {k: kind for k, (_, kind, _) in flat.nums.items()}
    mscales = {k: sc for k, (_, _, sc) in flat.nums.items()}
    ds = make_datasource(name, flat.num_rows, flat.ship_day, 86_400_000, dim_ids, dicts, mdata, mkinds, mscales,
                         segment_granularity="month", query_granularity="day", partition=flat.rank,
                         num_partitions=flat.world)
    ds.shard_key = "lo_orderkey"
    ds.build_indexes(bitmap_max_card=bitmap_max_card)
    return ds


# ------------------------------------------------------------------------------- star schema / SQL
SCHEMAS = {
    "lineorder": [("lo_orderkey", "integer"), ("lo_linenumber", "integer"), ("lo_custkey", "integer"),
                  ("lo_partkey", "integer"), ("lo_suppkey", "integer"), ("lo_orderdate", "integer"),
                  ("lo_orderpriority", "string"), ("lo_shippriority", "integer"), ("lo_quantity", "integer"),
                  ("lo_extendedprice", "bigint"), ("lo_ordtotalprice", "bigint"), ("lo_discount", "integer"),
                  ("lo_revenue", "bigint"), ("lo_supplycost", "bigint"), ("lo_tax", "integer"),
                  ("lo_commitdate", "integer"), ("lo_shipmode", "string")],
    "customer": [("c_custkey", "integer"), ("c_name", "string"), ("c_address", "string"), ("c_city", "string"),
                 ("c_nation", "string"), ("c_region", "string"), ("c_phone", "string"), ("c_mktsegment", "string")],
    "supplier": [("s_suppkey", "integer"), ("s_name", "string"), ("s_address", "string"), ("s_city", "string"),
                 ("s_nation", "string"), ("s_region", "string"), ("s_phone", "string")],
    "part": [("p_partkey", "integer"), ("p_name", "string"), ("p_mfgr", "string"), ("p_category", "string"),
             ("p_brand1", "string"), ("p_color", "string"), ("p_type", "string"), ("p_size", "integer"),
             ("p_container", "string")],
    "dwdate": [("d_datekey", "integer"), ("d_date", "string"), ("d_dayofweek", "string"), ("d_month", "string"),
               ("d_year", "integer"), ("d_yearmonthnum", "integer"), ("d_yearmonth", "string"),
               ("d_daynuminweek", "integer"), ("d_daynuminmonth", "integer"), ("d_daynuminyear", "integer"),
               ("d_monthnuminyear", "integer"), ("d_weeknuminyear", "integer"), ("d_sellingseason", "string")],
}


def star_schema_json(fact: str = "lineorder") -> str:
    def rel(r, a, b):
        return {"leftTable": fact, "rightTable": r, "relationType": "n-1",
                "joinCondition": [{"leftAttribute": a, "rightAttribute": b}]}
    return json.dumps({"factTable": fact, "relations": [
        rel("dwdate", "lo_orderdate", "d_datekey"), rel("customer", "lo_custkey", "c_custkey"),
        rel("supplier", "lo_suppkey", "s_suppkey"), rel("part", "lo_partkey", "p_partkey")]})


def ddl(table: str = "lineorder", source: str = "lineorderbase", datasource: str = "ssb",
        extra_options: str = "") -> str:
    ss = star_schema_json(table)
    return (f"CREATE TABLE if not exists {table} USING org.sparklinedata.druid OPTIONS ("
            f"sourceDataframe \"{source}\", timeDimensionColumn \"lo_orderdate\", druidDatasource \"{datasource}\", "
            f"druidHost 'localhost', allowTopNRewrite \"true\", starSchema '{ss}'{extra_options})")


def register(session, flat: Optional[FlatTPCH] = None, with_data: bool = False, table: str = "lineorder") -> None:
    """Register the SSB base tables (schema only, or with data for correctness checks) + the Druid
    star-schema fact table."""
    tabs = base_tables(flat) if with_data else {}
    session.register_table("lineorderbase", tabs.get("lineorder"), schema=SCHEMAS["lineorder"])
    for t in ("customer", "supplier", "part", "dwdate"):
        session.register_table(t, tabs.get(t), schema=SCHEMAS[t])
    session.sql(ddl(table))


def base_tables(flat: FlatTPCH) -> Dict[str, "object"]:
    """The SSB tables as pandas frames (small SF only): lineorder from the generated rows,
    dimension tables from the key -> attribute hashes."""
    import pandas as pd

    n = flat.num_rows

    def dec(name):
        d, ids = flat.dims[name]
        return d.decode(ids[:n].cpu().numpy().astype(np.int64))

    def numv(name):
        return flat.nums[name][0][:n].cpu().numpy().astype(np.int64)

    od = flat.ship_day.cpu().numpy().astype(np.int64)
    da = _date_attrs(START_DAY, END_DAY)
    datekey = np.asarray(da["d_datekey"], dtype=np.int64)[od - START_DAY]
    lo = pd.DataFrame({
        "lo_orderkey": dec("lo_orderkey"), "lo_linenumber": np.ones(n, dtype=np.int64),
        "lo_custkey": dec("lo_custkey"), "lo_partkey": dec("lo_partkey"), "lo_suppkey": dec("lo_suppkey"),
        "lo_orderdate": datekey, "lo_orderpriority": dec("lo_orderpriority"),
        "lo_shippriority": np.zeros(n, dtype=np.int64), "lo_quantity": dec("lo_quantity"),
        "lo_extendedprice": numv("lo_extendedprice"), "lo_ordtotalprice": numv("lo_ordtotalprice"),
        "lo_discount": dec("lo_discount"), "lo_revenue": numv("lo_revenue"), "lo_supplycost": numv("lo_supplycost"),
        "lo_tax": dec("lo_tax"), "lo_commitdate": datekey, "lo_shipmode": dec("lo_shipmode")})

    def dimtab(key, cols, extra):
        keys = np.asarray(dec(key.replace("c_custkey", "lo_custkey").replace("s_suppkey", "lo_suppkey")
                              .replace("p_partkey", "lo_partkey")))
        df = pd.DataFrame({key: keys, **{c: dec(c) for c in cols}}).drop_duplicates(key)
        for c, f in extra.items():
            df[c] = f(df)
        return df.reset_index(drop=True)

    cust = dimtab("c_custkey", ["c_name", "c_city", "c_nation", "c_region", "c_mktsegment"],
                  {"c_address": lambda d: "caddr-" + d.c_custkey.astype(str),
                   "c_phone": lambda d: "cphone-" + d.c_custkey.astype(str)})
    supp = dimtab("s_suppkey", ["s_name", "s_city", "s_nation", "s_region"],
                  {"s_address": lambda d: "saddr-" + d.s_suppkey.astype(str),
                   "s_phone": lambda d: "sphone-" + d.s_suppkey.astype(str)})
    part = dimtab("p_partkey", ["p_name", "p_mfgr", "p_category", "p_brand1", "p_color", "p_type", "p_size",
                                "p_container"], {})
    dw = pd.DataFrame(da)
    return {"lineorder": lo, "customer": cust[[c for c, _ in SCHEMAS["customer"]]],
            "supplier": supp[[c for c, _ in SCHEMAS["supplier"]]], "part": part[[c for c, _ in SCHEMAS["part"]]],
            "dwdate": dw[[c for c, _ in SCHEMAS["dwdate"]]]}


_J = "lineorder, dwdate"
QUERIES: List[Tuple[str, str]] = [
    ("Q1.1", f"""select sum(lo_extendedprice * lo_discount) as revenue from {_J}
        where lo_orderdate = d_datekey and d_year = 1993 and lo_discount between 1 and 3 and lo_quantity < 25"""),
    ("Q1.2", f"""select sum(lo_extendedprice * lo_discount) as revenue from {_J}
        where lo_orderdate = d_datekey and d_yearmonthnum = 199401 and lo_discount between 4 and 6
          and lo_quantity between 26 and 35"""),
    ("Q1.3", f"""select sum(lo_extendedprice * lo_discount) as revenue from {_J}
        where lo_orderdate = d_datekey and d_weeknuminyear = 6 and d_year = 1994 and lo_discount between 5 and 7
          and lo_quantity between 26 and 35"""),
    ("Q2.1", """select sum(lo_revenue) as lo_revenue, d_year, p_brand1 from lineorder, dwdate, part, supplier
        where lo_orderdate = d_datekey and lo_partkey = p_partkey and lo_suppkey = s_suppkey
          and p_category = 'MFGR#12' and s_region = 'AMERICA'
        group by d_year, p_brand1 order by d_year, p_brand1"""),
    ("Q2.2", """select sum(lo_revenue) as lo_revenue, d_year, p_brand1 from lineorder, dwdate, part, supplier
        where lo_orderdate = d_datekey and lo_partkey = p_partkey and lo_suppkey = s_suppkey
          and p_brand1 between 'MFGR#2221' and 'MFGR#2228' and s_region = 'ASIA'
        group by d_year, p_brand1 order by d_year, p_brand1"""),
    ("Q2.3", """select sum(lo_revenue) as lo_revenue, d_year, p_brand1 from lineorder, dwdate, part, supplier
        where lo_orderdate = d_datekey and lo_partkey = p_partkey and lo_suppkey = s_suppkey
          and p_brand1 = 'MFGR#2239' and s_region = 'EUROPE'
        group by d_year, p_brand1 order by d_year, p_brand1"""),
    ("Q3.1", """select c_nation, s_nation, d_year, sum(lo_revenue) as lo_revenue
        from customer, lineorder, supplier, dwdate
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_orderdate = d_datekey
          and c_region = 'ASIA' and s_region = 'ASIA' and d_year >= 1992 and d_year <= 1997
        group by c_nation, s_nation, d_year order by d_year asc, lo_revenue desc"""),
    ("Q3.2", """select c_city, s_city, d_year, sum(lo_revenue) as lo_revenue
        from customer, lineorder, supplier, dwdate
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_orderdate = d_datekey
          and c_nation = 'UNITED STATES' and s_nation = 'UNITED STATES' and d_year >= 1992 and d_year <= 1997
        group by c_city, s_city, d_year order by d_year asc, lo_revenue desc"""),
    ("Q3.3", """select c_city, s_city, d_year, sum(lo_revenue) as lo_revenue
        from customer, lineorder, supplier, dwdate
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_orderdate = d_datekey
          and (c_city = 'UNITED KI1' or c_city = 'UNITED KI5') and (s_city = 'UNITED KI1' or s_city = 'UNITED KI5')
          and d_year >= 1992 and d_year <= 1997
        group by c_city, s_city, d_year order by d_year asc, lo_revenue desc"""),
    ("Q3.4", """select c_city, s_city, d_year, sum(lo_revenue) as lo_revenue
        from customer, lineorder, supplier, dwdate
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_orderdate = d_datekey
          and (c_city = 'UNITED KI1' or c_city = 'UNITED KI5') and (s_city = 'UNITED KI1' or s_city = 'UNITED KI5')
          and d_yearmonth = 'Dec1997'
        group by c_city, s_city, d_year order by d_year asc, lo_revenue desc"""),
    ("Q4.1", """select d_year, c_nation, sum(lo_revenue - lo_supplycost) as profit
        from dwdate, customer, supplier, part, lineorder
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_partkey = p_partkey
          and lo_orderdate = d_datekey and c_region = 'AMERICA' and s_region = 'AMERICA'
          and (p_mfgr = 'MFGR#1' or p_mfgr = 'MFGR#2')
        group by d_year, c_nation order by d_year, c_nation"""),
    ("Q4.2", """select d_year, s_nation, p_category, sum(lo_revenue - lo_supplycost) as profit
        from dwdate, customer, supplier, part, lineorder
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_partkey = p_partkey
          and lo_orderdate = d_datekey and c_region = 'AMERICA' and s_region = 'AMERICA'
          and (d_year = 1997 or d_year = 1998) and (p_mfgr = 'MFGR#1' or p_mfgr = 'MFGR#2')
        group by d_year, s_nation, p_category order by d_year, s_nation, p_category"""),
    ("Q4.3", """select d_year, s_city, p_brand1, sum(lo_revenue - lo_supplycost) as profit
        from dwdate, customer, supplier, part, lineorder
        where lo_custkey = c_custkey and lo_suppkey = s_suppkey and lo_partkey = p_partkey
          and lo_orderdate = d_datekey and s_nation = 'UNITED STATES' and (d_year = 1997 or d_year = 1998)
          and p_category = 'MFGR#14'
        group by d_year, s_city, p_brand1 order by d_year, s_city, p_brand1"""),
]
# BASELINE config 4 additions: topN over a dictionary-encoded dimension and HLL count-distinct
EXTRA_QUERIES: List[Tuple[str, str]] = [
    ("TopN brand", """select p_brand1, sum(lo_revenue) as rev from lineorder, part
        where lo_partkey = p_partkey and p_mfgr = 'MFGR#1' group by p_brand1 order by rev desc limit 20"""),
    ("TopN city", """select c_city, sum(lo_revenue) as rev from lineorder, customer, dwdate
        where lo_custkey = c_custkey and lo_orderdate = d_datekey and d_year = 1997
        group by c_city order by rev desc limit 10"""),
    ("HLL customers", """select c_region, d_year, approx_count_distinct(lo_custkey) as custs
        from lineorder, customer, dwdate where lo_custkey = c_custkey and lo_orderdate = d_datekey
        group by c_region, d_year"""),
    ("HLL suppliers", """select p_category, approx_count_distinct(lo_suppkey) as supps
        from lineorder, part where lo_partkey = p_partkey and p_mfgr = 'MFGR#3' group by p_category"""),
]
ALL_QUERIES = QUERIES + EXTRA_QUERIES
