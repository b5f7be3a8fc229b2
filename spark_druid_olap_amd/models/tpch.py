"""TPC-H model family: the flattened ``orderLineItemPartSupplier`` table of the reference's
benchmark (``sd/tools/TpchBenchMark.scala:43-97``), its Druid index spec
(``src/test/resources/tpch_index_task.json.template:70-172``), DDL, star schema
(``tc/BaseTest.scala:29-141``), and the 8 benchmark queries (``TpchBenchMark.scala:135-292``).

Data is synthetic (BASELINE.json: "synthetic TPC-H data with random dictionary values") and is
generated ON THE DEVICE with torch in a few seconds even at SF100 (600M rows per GPU):
dbgen-like distributions and correlations (ship/commit/receipt dates derived from the order
date, return flag / line status from the 1995-06-17 "current date", extended price from the
part's retail price, order status / total price aggregated from the lines), with dimension
attributes computed from keys by integer hashing so every rank derives identical
customer/part/supplier attributes without materializing those tables.  For weak scaling each
rank owns a contiguous o_orderkey range (the shard key), so group-bys on o_orderkey never need
a cross-GPU merge.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..query.intervals import civil_from_days, days_from_civil
from ..segment.datasource import DataSource, make_datasource
from ..segment.dictionary import LONG, STRING, DOUBLE, Dictionary, FormattedDictionary, RangeDictionary, WordsDictionary

NATIONS = [("ALGERIA", 0), ("ARGENTINA", 1), ("BRAZIL", 1), ("CANADA", 1), ("EGYPT", 4), ("ETHIOPIA", 0),
           ("FRANCE", 3), ("GERMANY", 3), ("INDIA", 2), ("INDONESIA", 2), ("IRAN", 4), ("IRAQ", 4), ("JAPAN", 2),
           ("JORDAN", 4), ("KENYA", 0), ("MOROCCO", 0), ("MOZAMBIQUE", 0), ("PERU", 1), ("CHINA", 2),
           ("ROMANIA", 3), ("SAUDI ARABIA", 4), ("VIETNAM", 2), ("RUSSIA", 3), ("UNITED KINGDOM", 3),
           ("UNITED STATES", 1)]
REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
SEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
PRIORITIES = ["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"]
INSTRUCT = ["COLLECT COD", "DELIVER IN PERSON", "NONE", "TAKE BACK RETURN"]
SHIPMODES = ["AIR", "FOB", "MAIL", "RAIL", "REG AIR", "SHIP", "TRUCK"]
TYPE_S1 = ["STANDARD", "SMALL", "MEDIUM", "LARGE", "ECONOMY", "PROMO"]
TYPE_S2 = ["ANODIZED", "BURNISHED", "PLATED", "POLISHED", "BRUSHED"]
TYPE_S3 = ["TIN", "NICKEL", "BRASS", "STEEL", "COPPER"]
CONT_S1 = ["SM", "LG", "MED", "JUMBO", "WRAP"]
CONT_S2 = ["CASE", "BOX", "BAG", "JAR", "PKG", "PACK", "CAN", "DRUM"]

# TPC-H 4.2.3: the 92 part-name colours (p_name = 5 of them)
P_NAME_WORDS = [
    "almond", "antique", "aquamarine", "azure", "beige", "bisque", "black", "blanched", "blue", "blush", "brown",
    "burlywood", "burnished", "chartreuse", "chiffon", "chocolate", "coral", "cornflower", "cornsilk", "cream",
    "cyan", "dark", "deep", "dim", "dodger", "drab", "firebrick", "floral", "forest", "frosted", "gainsboro",
    "ghost", "goldenrod", "green", "grey", "honeydew", "hot", "indian", "ivory", "khaki", "lace", "lavender",
    "lawn", "lemon", "light", "lime", "linen", "magenta", "maroon", "medium", "metallic", "midnight", "mint",
    "misty", "moccasin", "navajo", "navy", "olive", "orange", "orchid", "pale", "papaya", "peach", "peru", "pink",
    "plum", "powder", "puff", "purple", "red", "rose", "rosy", "royal", "saddle", "salmon", "sandy", "seashell",
    "sienna", "sky", "slate", "smoke", "snow", "spring", "steel", "tan", "thistle", "tomato", "turquoise",
    "violet", "wheat", "white", "yellow"]
# comment text: a slice of the TPC-H 4.2.2.10 text-grammar vocabulary (nouns, verbs, adjectives,
# adverbs, prepositions) including the words Q13 / Q16 look for
COMMENT_WORDS = [
    "foxes", "ideas", "theodolites", "pinto", "beans", "instructions", "dependencies", "excuses", "platelets",
    "asymptotes", "courts", "dolphins", "packages", "requests", "accounts", "deposits", "sleep", "wake", "are",
    "cajole", "haggle", "nag", "use", "boost", "affix", "detect", "integrate", "furious", "sly", "careful",
    "blithe", "quick", "fluffy", "slow", "quiet", "ruthless", "thin", "close", "regular", "special", "pending",
    "unusual", "express", "final", "ironic", "even", "bold", "silent", "about", "above", "according", "across",
    "after", "against", "along", "among", "around", "Customer", "Complaints", "Recommends"]

START_DAY = days_from_civil(1992, 1, 1)
CURRENT_DAY = days_from_civil(1995, 6, 17)
ORDER_SPAN = 2406  # orderdate in [1992-01-01, 1998-08-02]
DATE_DICT_END = days_from_civil(1999, 12, 31)

# Druid index spec (tpch_index_task.json.template:70-108 dims, 114-172 metrics)
INDEX_DIMS = ["o_orderkey", "o_orderdate", "o_orderstatus", "o_orderpriority", "o_clerk", "o_shippriority",
              "o_comment", "l_returnflag", "l_linestatus", "l_commitdate", "l_receiptdate", "l_shipinstruct",
              "l_shipmode", "l_comment", "ps_comment", "s_name", "s_address", "s_phone", "s_comment",
              "s_nation", "s_region", "p_name", "p_mfgr", "p_brand", "p_type", "p_size", "p_container",
              "p_retailprice", "p_comment", "c_name", "c_address", "c_phone", "c_mktsegment", "c_comment",
              "c_nation", "c_region"]
# metric name -> (source expression, kind, scale)
INDEX_METRICS = {
    "o_totalprice": ("o_totalprice", "decimal", 2),
    "sum_l_quantity": ("l_quantity", "long", 0),
    "l_extendedprice": ("l_extendedprice", "decimal", 2),
    "l_tax": ("js_l_tax", "decimal", 6),             # ext * (1 - disc) * tax
    "l_discount": ("js_l_discount", "decimal", 4),   # ext * disc
    "sum_ps_availqty": ("ps_availqty", "long", 0),
    "ps_supplycost": ("ps_supplycost", "decimal", 2),
    "c_acctbal": ("c_acctbal", "decimal", 2),
}

# The benchmark index (docs/benchmark/druid/tpch_index.json): raw-grain, metric names == SQL names.
BENCH_INDEX_DIMS = ["o_orderkey", "o_custkey", "o_orderdate", "o_orderstatus", "o_orderpriority", "o_clerk",
                    "o_shippriority", "o_comment", "l_partkey", "l_suppkey", "l_linenumber", "l_returnflag",
                    "l_linestatus", "l_commitdate", "l_receiptdate", "l_shipinstruct", "l_shipmode", "l_comment",
                    "ps_comment", "s_name", "s_address", "s_phone", "s_acctbal", "s_comment", "s_nation", "s_region", "p_name",
                    "p_mfgr", "p_brand", "p_type", "p_container", "p_comment", "c_name", "c_address", "c_phone",
                    "c_mktsegment", "c_comment", "c_nation", "c_region"]
BENCH_INDEX_METRICS = {
    "o_totalprice": ("o_totalprice", "decimal", 2),
    "l_quantity": ("l_quantity", "long", 0),
    "l_extendedprice": ("l_extendedprice", "decimal", 2),
    "l_discount": ("l_discount", "decimal", 2),
    "l_tax": ("l_tax", "decimal", 2),
    "ps_availqty": ("ps_availqty", "long", 0),
    "ps_supplycost": ("ps_supplycost", "decimal", 2),
    "p_size": ("p_size_m", "long", 0),
    "p_retailprice": ("p_retailprice_m", "decimal", 2),
    "c_acctbal": ("c_acctbal", "decimal", 2),
}

FLAT_SCHEMA = [
    ("o_orderkey", "integer"), ("o_custkey", "integer"), ("o_orderstatus", "string"), ("o_totalprice", "double"),
    ("o_orderdate", "string"), ("o_orderpriority", "string"), ("o_clerk", "string"), ("o_shippriority", "integer"),
    ("o_comment", "string"), ("l_partkey", "integer"), ("l_suppkey", "integer"), ("l_linenumber", "integer"),
    ("l_quantity", "double"), ("l_extendedprice", "double"), ("l_discount", "double"), ("l_tax", "double"),
    ("l_returnflag", "string"), ("l_linestatus", "string"), ("l_shipdate", "string"), ("l_commitdate", "string"),
    ("l_receiptdate", "string"), ("l_shipinstruct", "string"), ("l_shipmode", "string"), ("l_comment", "string"),
    ("order_year", "string"), ("ps_partkey", "integer"), ("ps_suppkey", "integer"), ("ps_availqty", "integer"),
    ("ps_supplycost", "double"), ("ps_comment", "string"), ("s_name", "string"), ("s_address", "string"),
    ("s_phone", "string"), ("s_acctbal", "double"), ("s_comment", "string"), ("s_nation", "string"),
    ("s_region", "string"), ("p_name", "string"), ("p_mfgr", "string"), ("p_brand", "string"), ("p_type", "string"),
    ("p_size", "integer"), ("p_container", "string"), ("p_retailprice", "double"), ("p_comment", "string"),
    ("c_name", "string"), ("c_address", "string"), ("c_phone", "string"), ("c_acctbal", "double"),
    ("c_mktsegment", "string"), ("c_comment", "string"), ("c_nation", "string"), ("c_region", "string"),
]

COLUMN_MAPPING = {"l_quantity": "sum_l_quantity", "ps_availqty": "sum_ps_availqty", "cn_name": "c_nation",
                  "cr_name": "c_region", "sn_name": "s_nation", "sr_name": "s_region"}

FUNCTIONAL_DEPENDENCIES = [
    {"col1": "c_name", "col2": "c_address", "type": "1-1"},
    {"col1": "c_phone", "col2": "c_address", "type": "1-1"},
    {"col1": "c_name", "col2": "c_mktsegment", "type": "n-1"},
    {"col1": "c_name", "col2": "c_comment", "type": "1-1"},
    {"col1": "c_name", "col2": "c_nation", "type": "n-1"},
    {"col1": "c_nation", "col2": "c_region", "type": "n-1"},
]


def date_strings(d0: int, d1: int) -> List[str]:
    out = []
    for d in range(d0, d1 + 1):
        y, m, dd = civil_from_days(d)
        out.append(f"{y:04d}-{m:02d}-{dd:02d}")
    return out


def _sorted_codes(values: List[str]) -> Tuple[Dictionary, np.ndarray]:
    """dictionary sorted lexicographically + map from generation index -> sorted id"""
    order = sorted(range(len(values)), key=lambda i: values[i])
    d = Dictionary([values[i] for i in order], STRING)
    remap = np.empty(len(values), dtype=np.int64)
    for sid, i in enumerate(order):
        remap[i] = sid
    return d, remap


_C1 = 0x9E3779B97F4A7C15 - (1 << 64)
_C2 = 0xBF58476D1CE4E5B9 - (1 << 64)
_C3 = 0x94D049BB133111EB - (1 << 64)


def _lsr(x, s):
    return (x >> s) & ((1 << (64 - s)) - 1)


def khash(x: torch.Tensor, salt: int) -> torch.Tensor:
    """splitmix64 of (key, salt): deterministic per-key attributes, non-negative int64."""
    add = ((salt * 0x9E3779B97F4A7C15 + (1 << 63)) % (1 << 64)) - (1 << 63)
    z = x.to(torch.int64) * 0x10001 + add
    z = (z ^ _lsr(z, 30)) * _C2
    z = (z ^ _lsr(z, 27)) * _C3
    z = z ^ _lsr(z, 31)
    return z & ((1 << 62) - 1)


@dataclass
class FlatTPCH:
    """Column-oriented flattened TPC-H rows (time-sorted by l_shipdate) on one device."""
    sf: float
    rank: int
    world: int
    num_rows: int
    ship_day: torch.Tensor                       # int32 days since epoch (sorted)
    dims: Dict[str, Tuple[Dictionary, torch.Tensor]] = field(default_factory=dict)
    nums: Dict[str, Tuple[torch.Tensor, str, int]] = field(default_factory=dict)  # tensor, kind, scale
    counts: Dict[str, int] = field(default_factory=dict)


def _bijection(x: torch.Tensor, n: int, salt: int) -> torch.Tensor:
    """x -> (a x + b) mod n, a permutation of [0, n) (a coprime with n): scatters entity keys over
    a phrase dictionary so the leading words do not track the key order."""
    for a in (1_000_003, 999_983, 1_000_033, 998_999, 1_000_037):
        if math.gcd(a, n) == 1:
            break
    return torch.remainder(x.to(torch.int64) * a + salt * 7_919, n)


def generate_flat(sf: float = 1.0, device="cpu", rank: int = 0, world: int = 1, seed: int = 20260101,
                  columns: Optional[List[str]] = None) -> FlatTPCH:
    """Generate this rank's share of a TPC-H SF (per-rank) flattened table on `device`."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed * 1000 + rank)
    No = max(8, int(round(1_500_000 * sf)))
    tot_orders = No * world
    C = max(10, int(round(150_000 * sf * world)))
    P = max(20, int(round(200_000 * sf * world)))
    Sn = max(4, int(round(10_000 * sf * world)))
    clerks = max(1, int(round(1000 * sf * world)))

    def rint(lo, hi, n, dtype=torch.int32):
        return torch.randint(lo, hi, (n,), generator=g, device=dev, dtype=dtype)

    orderkey = torch.arange(No, device=dev, dtype=torch.int64) + rank * No + 1
    odate = rint(0, ORDER_SPAN, No) + START_DAY                  # int32 days
    custkey = rint(1, C + 1, No, torch.int64)
    opri = rint(0, 5, No, torch.int16)
    clerk = rint(0, clerks, No)
    nlines = rint(1, 8, No, torch.int64)
    L = int(nlines.sum().item())
    oidx = torch.repeat_interleave(torch.arange(No, device=dev, dtype=torch.int64), nlines)
    first = torch.cumsum(nlines, 0) - nlines
    linenum = (torch.arange(L, device=dev, dtype=torch.int64) - torch.repeat_interleave(first, nlines) + 1).to(torch.int8)
    partkey = rint(1, P + 1, L, torch.int64)
    supp_i = rint(0, 4, L, torch.int64)
    suppkey = (partkey + supp_i * (Sn // 4 + (partkey - 1) // Sn)) % Sn + 1
    qty = rint(1, 51, L, torch.int16)
    retail = 90000 + torch.remainder(partkey // 10, 20001) + 100 * torch.remainder(partkey, 1000)  # cents
    ext = qty.to(torch.int64) * retail                                       # cents
    disc = rint(0, 11, L, torch.int16)                                       # percent
    tax = rint(0, 9, L, torch.int16)
    od_l = odate[oidx]
    ship = od_l + rint(1, 122, L)
    commit = od_l + rint(30, 91, L)
    receipt = ship + rint(1, 31, L)
    rflag_ra = rint(0, 2, L, torch.int8)
    # A=0, N=1, R=2
    rflag = torch.where(receipt <= CURRENT_DAY, torch.where(rflag_ra == 0, 0, 2), 1).to(torch.uint8)
    lstatus = (ship > CURRENT_DAY).to(torch.uint8)                          # F=0, O=1
    instr = rint(0, 4, L, torch.uint8)
    smode = rint(0, 7, L, torch.uint8)
    # order status & total price aggregated from the lines
    ocnt_o = torch.zeros(No, dtype=torch.int64, device=dev).index_add_(0, oidx, lstatus.to(torch.int64))
    ostatus = torch.where(ocnt_o == 0, 0, torch.where(ocnt_o == nlines, 1, 2)).to(torch.uint8)  # F, O, P
    line_total = ext * (100 + tax.to(torch.int64)) * (100 - disc.to(torch.int64))  # cents * 1e4
    ototal = torch.zeros(No, dtype=torch.int64, device=dev).index_add_(0, oidx, line_total)
    ototal = torch.div(ototal + 5000, 10000, rounding_mode="floor")          # cents

    # ---- sort the lines by ship date (the Druid time dimension) ----
    perm = torch.argsort(ship, stable=True)
    del first
    ship = ship[perm]

    def P_(t):
        return t[perm]

    oidx = P_(oidx)
    line_cols = {"partkey": P_(partkey), "supp_i": P_(supp_i), "suppkey": P_(suppkey), "qty": P_(qty),
                 "ext": P_(ext), "disc": P_(disc), "tax": P_(tax), "commit": P_(commit), "receipt": P_(receipt),
                 "rflag": P_(rflag), "lstatus": P_(lstatus), "instr": P_(instr), "smode": P_(smode),
                 "linenum": P_(linenum)}
    del partkey, supp_i, suppkey, qty, ext, disc, tax, commit, receipt, rflag, lstatus, instr, smode, linenum, perm

    flat = FlatTPCH(sf, rank, world, L, ship.to(torch.int32))
    flat.counts = {"orders": tot_orders, "customers": C, "parts": P, "suppliers": Sn, "clerks": clerks}
    want = set(columns) if columns else None

    def need(name):
        return want is None or name in want

    def dim(name, d, ids):
        if need(name):
            flat.dims[name] = (d, ids)

    def num(name, t, kind, scale=0):
        if need(name):
            flat.nums[name] = (t, kind, scale)

    date_d = Dictionary(date_strings(START_DAY, DATE_DICT_END), STRING)
    ok_l = orderkey[oidx]
    pk = line_cols["partkey"]
    sk = line_cols["suppkey"]
    ck = custkey[oidx]
    nat_d, nat_remap = _sorted_codes([n for n, _ in NATIONS])
    nat_remap_t = torch.from_numpy(nat_remap).to(dev)
    reg_of_nation = torch.tensor([r for _, r in NATIONS], device=dev, dtype=torch.int64)
    reg_d = Dictionary(REGIONS, STRING)

    # orders
    dim("o_orderkey", RangeDictionary(1, tot_orders), (ok_l - 1).to(torch.int32))
    num("o_custkey", ck.to(torch.int32), "long")
    dim("o_orderstatus", Dictionary(["F", "O", "P"]), ostatus[oidx])
    num("o_totalprice", ototal[oidx].to(torch.int32) if ototal.numel() and int(ototal.max()) < 2 ** 31 else ototal[oidx], "decimal", 2)
    dim("o_orderdate", date_d, (odate[oidx] - START_DAY).to(torch.int16))
    dim("o_orderpriority", Dictionary(PRIORITIES), opri[oidx].to(torch.uint8))
    dim("o_clerk", FormattedDictionary("Clerk#", 9, clerks, start=1), clerk[oidx])
    dim("o_shippriority", Dictionary([0], LONG), torch.zeros(L, dtype=torch.uint8, device=dev))
    dim("o_comment", WordsDictionary(COMMENT_WORDS, 6, tot_orders), _bijection(ok_l - 1, tot_orders, 1).to(torch.int32))
    # lineitem
    num("l_partkey", pk.to(torch.int32), "long")
    num("l_suppkey", sk.to(torch.int32), "long")
    num("l_linenumber", line_cols["linenum"].to(torch.int16), "long")
    if need("l_partkey"):
        flat.dims["l_partkey"] = (RangeDictionary(1, P), (pk - 1).to(torch.int32))
        flat.dims["l_suppkey"] = (RangeDictionary(1, Sn), (sk - 1).to(torch.int32))
        flat.dims["l_linenumber"] = (Dictionary(list(range(1, 8)), LONG), (line_cols["linenum"] - 1).to(torch.uint8))
    if need("o_custkey"):
        flat.dims["o_custkey"] = (RangeDictionary(1, C), (ck - 1).to(torch.int32))
    num("l_quantity", line_cols["qty"], "long")
    num("l_extendedprice", line_cols["ext"].to(torch.int32), "decimal", 2)
    num("l_discount", line_cols["disc"], "decimal", 2)
    num("l_tax", line_cols["tax"], "decimal", 2)
    dim("l_returnflag", Dictionary(["A", "N", "R"]), line_cols["rflag"])
    dim("l_linestatus", Dictionary(["F", "O"]), line_cols["lstatus"])
    dim("l_commitdate", date_d, (line_cols["commit"] - START_DAY).to(torch.int16))
    dim("l_receiptdate", date_d, (line_cols["receipt"] - START_DAY).to(torch.int16))
    dim("l_shipinstruct", Dictionary(INSTRUCT), line_cols["instr"])
    dim("l_shipmode", Dictionary(SHIPMODES), line_cols["smode"])
    lc_n = tot_orders * 8
    if lc_n < 2 ** 31:
        dim("l_comment", FormattedDictionary("lcomment-", 11, lc_n), ((ok_l - 1) * 8 + line_cols["linenum"].to(torch.int64)).to(torch.int32))
    # index-time javascript metrics (exact decimals)
    ext64 = line_cols["ext"]
    d64 = line_cols["disc"].to(torch.int64)
    t64 = line_cols["tax"].to(torch.int64)
    num("js_l_tax", ext64 * (100 - d64) * t64, "decimal", 6)
    num("js_l_discount", (ext64 * d64).to(torch.int32), "decimal", 4)
    # partsupp
    psid = (pk - 1) * 4 + line_cols["supp_i"]
    num("ps_partkey", pk.to(torch.int32), "long")
    num("ps_suppkey", sk.to(torch.int32), "long")
    num("ps_availqty", (khash(psid, 10) % 9999 + 1).to(torch.int16), "long")
    num("ps_supplycost", (khash(psid, 11) % 99901 + 100).to(torch.int32), "decimal", 2)
    dim("ps_comment", FormattedDictionary("pscomment-", 10, P * 4), psid.to(torch.int32))
    # supplier
    s_nk = khash(sk, 9) % 25
    dim("s_name", FormattedDictionary("Supplier#", 9, Sn, start=1), (sk - 1).to(torch.int32))
    dim("s_address", FormattedDictionary("saddr-", 9, Sn, start=1), (sk - 1).to(torch.int32))
    dim("s_phone", FormattedDictionary("sphone-", 9, Sn, start=1), (sk - 1).to(torch.int32))
    num("s_acctbal", (khash(sk, 12) % 1099999 - 99999).to(torch.int32), "decimal", 2)
    dim("s_comment", WordsDictionary(COMMENT_WORDS, 6, Sn), _bijection(sk - 1, Sn, 2).to(torch.int32))
    dim("s_nation", nat_d, nat_remap_t[s_nk].to(torch.uint8))
    dim("s_region", reg_d, reg_of_nation[s_nk].to(torch.uint8))
    # part
    types = [f"{a} {b} {c}" for a in TYPE_S1 for b in TYPE_S2 for c in TYPE_S3]
    type_d, type_remap = _sorted_codes(types)
    conts = [f"{a} {b}" for a in CONT_S1 for b in CONT_S2]
    cont_d, cont_remap = _sorted_codes(conts)
    mfgr = khash(pk, 5) % 5
    dim("p_name", WordsDictionary(P_NAME_WORDS, 5, P), _bijection(pk - 1, P, 3).to(torch.int32))
    dim("p_mfgr", Dictionary([f"Manufacturer#{i}" for i in range(1, 6)]), mfgr.to(torch.uint8))
    dim("p_brand", Dictionary([f"Brand#{i}{j}" for i in range(1, 6) for j in range(1, 6)]),
        (mfgr * 5 + khash(pk, 6) % 5).to(torch.uint8))
    dim("p_type", type_d, torch.from_numpy(type_remap).to(dev)[khash(pk, 4) % 150].to(torch.uint8))
    dim("p_size", Dictionary(list(range(1, 51)), LONG), (khash(pk, 7) % 50).to(torch.uint8))
    dim("p_container", cont_d, torch.from_numpy(cont_remap).to(dev)[khash(pk, 8) % 40].to(torch.uint8))
    retail_l = 90000 + torch.remainder(pk // 10, 20001) + 100 * torch.remainder(pk, 1000)
    dim("p_retailprice", Dictionary(np.arange(90000, 210000) / 100.0, DOUBLE), (retail_l - 90000).to(torch.int32))
    num("p_retailprice_m", retail_l.to(torch.int32), "decimal", 2)
    num("p_size_m", (khash(pk, 7) % 50 + 1).to(torch.int16), "long")
    dim("p_comment", FormattedDictionary("pcomment-", 9, P, start=1), (pk - 1).to(torch.int32))
    # customer
    c_nk = khash(ck, 1) % 25
    dim("c_name", FormattedDictionary("Customer#", 9, C, start=1), (ck - 1).to(torch.int32))
    dim("c_address", FormattedDictionary("caddr-", 9, C, start=1), (ck - 1).to(torch.int32))
    dim("c_phone", FormattedDictionary("cphone-", 9, C, start=1), (ck - 1).to(torch.int32))
    num("c_acctbal", (khash(ck, 3) % 1099999 - 99999).to(torch.int32), "decimal", 2)
    dim("c_mktsegment", Dictionary(SEGMENTS), (khash(ck, 2) % 5).to(torch.uint8))
    dim("c_comment", FormattedDictionary("ccomment-", 9, C, start=1), (ck - 1).to(torch.int32))
    dim("c_nation", nat_d, nat_remap_t[c_nk].to(torch.uint8))
    dim("c_region", reg_d, reg_of_nation[c_nk].to(torch.uint8))
    return flat


_NUM_ALIAS = {"ps_partkey": "l_partkey", "ps_suppkey": "l_suppkey"}


def _numeric_dim(t: torch.Tensor, scale: int):
    """Dictionary-encode a numeric column as a (string-valued, like Druid) dimension."""
    uniq, inv = torch.unique(t.to(torch.int64), return_inverse=True)
    vals = uniq.cpu().numpy()
    # typed (numeric-order) dictionary: bounds stay id ranges and values decode to numbers
    d = Dictionary(vals / 10 ** scale, DOUBLE) if scale else Dictionary(vals, LONG)
    from ..segment.dictionary import id_dtype_for

    return d, inv.to(getattr(torch, {"uint8": "uint8", "int16": "int16"}.get(id_dtype_for(len(vals)), "int32")))


def to_datasource(flat: FlatTPCH, name: str = "tpch", bitmap_max_card: int = 256,
                  bitmap_budget_bytes: Optional[int] = None, profile: str = "bench") -> DataSource:
    """Build the Druid-index datasource (index dims + index metrics) from the flat columns.

    profile "bench": docs/benchmark/druid/tpch_index.json (the published benchmark's index);
    profile "test": src/test/resources/tpch_index_task.json.template (the test-suite index)."""
    dims_l, mets = (BENCH_INDEX_DIMS, BENCH_INDEX_METRICS) if profile == "bench" else (INDEX_DIMS, INDEX_METRICS)
    if profile == "test":
        # the test index spells "dimension" (tpch_index_task.json.template:70), which Druid ignores:
        # dimensions are schemaless = every column but the timestamp and the metric names
        dims_l = [c for c, _ in FLAT_SCHEMA if c != "l_shipdate" and c not in mets]
    dim_ids, dicts = {}, {}
    for d in dims_l:
        if d in flat.dims:
            dicts[d], dim_ids[d] = flat.dims[d]
        elif d in flat.nums or d in _NUM_ALIAS:
            t, _, scale = flat.nums[_NUM_ALIAS.get(d, d)]
            dicts[d], dim_ids[d] = _numeric_dim(t, scale)
        elif d == "order_year" and "o_orderdate" in flat.dims:
            # the test index's order_year dimension (tpch_index_task.json.template:39): the year of
            # o_orderdate, one id per distinct year
            od_dict, od_ids = flat.dims["o_orderdate"]
            vals = [str(v)[:4] for v in od_dict.all_values()]
            years = sorted(set(vals))
            remap = torch.tensor([years.index(v) for v in vals], dtype=torch.int16, device=od_ids.device)
            dicts[d], dim_ids[d] = Dictionary(years, STRING), remap[od_ids.to(torch.int64)]
    mdata, mkinds, mscales = {}, {}, {}
    for mname, (src, kind, scale) in mets.items():
        if src in flat.nums:
            t, _, _ = flat.nums[src]
            mdata[mname], mkinds[mname], mscales[mname] = t, kind, scale
    ds = make_datasource(name, flat.num_rows, flat.ship_day, 86_400_000, dim_ids, dicts, mdata, mkinds, mscales,
                         segment_granularity="month", query_granularity="day", partition=flat.rank,
                         num_partitions=flat.world)
    ds.shard_key = "o_orderkey"
    ds.build_indexes(bitmap_max_card=bitmap_max_card, bitmap_budget_bytes=bitmap_budget_bytes)
    return ds


def to_pandas(flat: FlatTPCH, lo: int = 0, hi: Optional[int] = None):
    """The raw 53-column base table (`orderLineItemPartSupplierBase`) as a pandas DataFrame (rows
    ``[lo, hi)``; chunked export keeps host memory bounded at large scale factors)."""
    import pandas as pd

    n = flat.num_rows if hi is None else min(hi, flat.num_rows)
    out = {}
    ship = flat.ship_day[lo:n].cpu().numpy().astype(np.int64)
    date_d = Dictionary(date_strings(START_DAY, DATE_DICT_END), STRING)
    for name, typ in FLAT_SCHEMA:
        if name == "l_shipdate":
            out[name] = date_d.decode(ship - START_DAY)
        elif name == "order_year":
            od = flat.dims["o_orderdate"][1][lo:n].cpu().numpy().astype(np.int64)
            years = np.array([s[:4] for s in date_d.values], dtype=object)
            out[name] = years[od]
        elif name in flat.dims:
            d, ids = flat.dims[name]
            out[name] = d.decode(ids[lo:n].cpu().numpy().astype(np.int64))
        elif name in flat.nums:
            t, kind, scale = flat.nums[name]
            v = t[lo:n].cpu().numpy()
            if kind == "decimal":
                v = v.astype(np.float64) / (10.0 ** scale)
            elif typ == "double":
                v = v.astype(np.float64)
            out[name] = v
    df = pd.DataFrame(out, columns=[c for c, _ in FLAT_SCHEMA if c in out])
    return df


# --------------------------------------------------------------------------- DDL and queries
def druid_ddl(table: str = "orderLineItemPartSupplier", source: str = "orderLineItemPartSupplierBase",
              datasource: str = "tpch", extra_options: str = "", with_column_mapping: bool = True,
              star_schema: Optional[str] = None) -> str:
    """The reference's Druid DDL (``tc/BaseTest.scala:167-182``).  The benchmark index
    (``docs/benchmark/druid/tpch_index.json``) keeps SQL column names, so the bench passes
    ``with_column_mapping=False``."""
    import json

    cm = f"columnMapping '{json.dumps(COLUMN_MAPPING)}', " if with_column_mapping else ""
    ss = star_schema or f'{{"factTable" : "{table}", "relations" : []}}'
    return (f"CREATE TABLE if not exists {table} USING org.sparklinedata.druid OPTIONS ("
            f"sourceDataframe \"{source}\", timeDimensionColumn \"l_shipdate\", druidDatasource \"{datasource}\", "
            f"druidHost 'localhost', zkQualifyDiscoveryNames \"true\", "
            f"{cm}numProcessingThreadsPerHistorical '1', "
            f"allowTopNRewrite \"true\", functionalDependencies '{json.dumps(FUNCTIONAL_DEPENDENCIES)}', "
            f"starSchema '{ss}'{extra_options})")


T = "orderLineItemPartSupplier"

# The 8 queries of TpchBenchMark.scala:135-292 (dateTime(...) expressions written with the
# sparkline date UDF syntax supported by our SQL front-end).
BENCH_QUERIES: List[Tuple[str, str]] = [
    ("Basic Aggregation", f"""select l_returnflag, l_linestatus, count(*), sum(l_extendedprice) as s,
        max(ps_supplycost) as m, avg(ps_availqty) as a, count(distinct o_orderkey)
        from {T} group by l_returnflag, l_linestatus"""),
    ("Ship Date Range", f"""select f, s, count(*) as count_order from
        (select l_returnflag as f, l_linestatus as s, l_shipdate, s_region, s_nation, c_nation from {T}) t
        where dateIsBeforeOrEqual(dateTime(`l_shipdate`), dateMinus(dateTime("1997-12-01"), period("P90D")))
          and dateIsAfter(dateTime(`l_shipdate`), dateTime("1995-12-01"))
        group by f, s"""),
    ("SubQuery + nation,Type predicates + ShipDate Range", f"""select s_nation, count(*) as count_order,
        sum(l_extendedprice) as s, max(ps_supplycost) as m, avg(ps_availqty) as a, count(distinct o_orderkey)
        from (select l_returnflag as f, l_linestatus as s, l_shipdate, s_region, s_nation, c_nation, p_type,
                     l_extendedprice, ps_supplycost, ps_availqty, o_orderkey
              from {T} where p_type = 'ECONOMY ANODIZED STEEL') t
        where dateIsBeforeOrEqual(dateTime(`l_shipdate`), dateMinus(dateTime("1997-12-01"), period("P90D")))
          and dateIsAfter(dateTime(`l_shipdate`), dateTime("1995-12-01"))
          and ((s_nation = 'FRANCE' and c_nation = 'GERMANY') or (c_nation = 'FRANCE' and s_nation = 'GERMANY'))
        group by s_nation"""),
    ("TPCH Q1", f"""select l_returnflag, l_linestatus, count(*), sum(l_extendedprice) as s,
        max(ps_supplycost) as m, avg(ps_availqty) as a, count(distinct o_orderkey)
        from {T} group by l_returnflag, l_linestatus"""),
    ("TPCH Q3", f"""select o_orderkey, sum(l_extendedprice) as price, o_orderdate, o_shippriority
        from {T} where c_mktsegment = 'BUILDING'
          and dateIsBefore(dateTime(`o_orderdate`), dateTime("1995-03-15"))
          and dateIsAfter(dateTime(`l_shipdate`), dateTime("1995-03-15"))
        group by o_orderkey, o_orderdate, o_shippriority"""),
    ("TPCH Q5", f"""select s_nation, sum(l_extendedprice) as extendedPrice from {T}
        where s_region = 'ASIA'
          and dateIsAfterOrEqual(dateTime(`o_orderdate`), dateTime("1994-01-01"))
          and dateIsBefore(dateTime(`o_orderdate`), datePlus(dateTime("1994-01-01"), period("P1Y")))
        group by s_nation"""),
    ("TPCH Q7", f"""select s_nation, c_nation, year(dateTime(`l_shipdate`)) as l_year,
        sum(l_extendedprice) as extendedPrice from {T}
        where ((s_nation = 'FRANCE' and c_nation = 'GERMANY') or (c_nation = 'FRANCE' and s_nation = 'GERMANY'))
        group by s_nation, c_nation, year(dateTime(`l_shipdate`))"""),
    ("TPCH Q8", f"""select year(dateTime(`o_orderdate`)) as o_year, sum(l_extendedprice) as price from {T}
        where c_region = 'AMERICA' and p_type = 'ECONOMY ANODIZED STEEL'
          and dateIsAfterOrEqual(dateTime(`o_orderdate`), dateTime("1995-01-01"))
          and dateIsBeforeOrEqual(dateTime(`o_orderdate`), dateTime("1996-12-31"))
        group by year(dateTime(`o_orderdate`))"""),
]

Q10 = ("TPCH Q10", f"""select c_name, c_nation, c_address, c_phone, c_comment, sum(l_extendedprice) as price
    from {T}
    where dateIsAfterOrEqual(dateTime(`o_orderdate`), dateTime("1993-10-01"))
      and dateIsBefore(dateTime(`o_orderdate`), datePlus(dateTime("1993-10-01"), period("P3M")))
      and l_returnflag = 'R'
    group by c_name, c_nation, c_address, c_phone, c_comment""")


# --------------------------------------------------------------------------- star schema
# The reference's TPC-H star schema over the same denormalized index (tc/BaseTest.scala:59-141,
# documented at sd/metadata/StarSchemaInfo.scala:138-165): nation/region are split into customer-
# and supplier-side copies so every table has a unique join path and column names stay unique.
STAR_COLUMN_MAPPING = {"cn_name": "c_nation", "cr_name": "c_region", "sn_name": "s_nation", "sr_name": "s_region"}


def star_schema_json(fact_db: str = "default", dim_db: str = "default") -> str:
    import json

    def rel(l, r, keys):
        return {"leftTable": l, "rightTable": r, "relationType": "n-1",
                "joinCondition": [{"leftAttribute": a, "rightAttribute": b} for a, b in keys]}
    f, d = fact_db, dim_db
    rels = [rel(f"{f}.lineitem", f"{d}.orders", [("l_orderkey", "o_orderkey")]),
            rel(f"{f}.lineitem", f"{d}.partsupp", [("l_partkey", "ps_partkey"), ("l_suppkey", "ps_suppkey")]),
            rel(f"{d}.partsupp", f"{d}.part", [("ps_partkey", "p_partkey")]),
            rel(f"{d}.partsupp", f"{d}.supplier", [("ps_suppkey", "s_suppkey")]),
            rel(f"{d}.orders", f"{d}.customer", [("o_custkey", "c_custkey")]),
            rel(f"{d}.customer", f"{d}.custnation", [("c_nationkey", "cn_nationkey")]),
            rel(f"{d}.custnation", f"{d}.custregion", [("cn_regionkey", "cr_regionkey")]),
            rel(f"{d}.supplier", f"{d}.suppnation", [("s_nationkey", "sn_nationkey")]),
            rel(f"{d}.suppnation", f"{d}.suppregion", [("sn_regionkey", "sr_regionkey")])]
    return json.dumps({"factTable": f"{f}.lineitem", "relations": rels})


STAR_SCHEMAS = {
    "lineitembase": [("l_orderkey", "integer"), ("l_partkey", "integer"), ("l_suppkey", "integer"),
                     ("l_linenumber", "integer"), ("l_quantity", "double"), ("l_extendedprice", "double"),
                     ("l_discount", "double"), ("l_tax", "double"), ("l_returnflag", "string"),
                     ("l_linestatus", "string"), ("l_shipdate", "string"), ("l_commitdate", "string"),
                     ("l_receiptdate", "string"), ("l_shipinstruct", "string"), ("l_shipmode", "string"),
                     ("l_comment", "string")],
    "orders": [("o_orderkey", "integer"), ("o_custkey", "integer"), ("o_orderstatus", "string"),
               ("o_totalprice", "double"), ("o_orderdate", "string"), ("o_orderpriority", "string"),
               ("o_clerk", "string"), ("o_shippriority", "integer"), ("o_comment", "string")],
    "partsupp": [("ps_partkey", "integer"), ("ps_suppkey", "integer"), ("ps_availqty", "integer"),
                 ("ps_supplycost", "double"), ("ps_comment", "string")],
    "part": [("p_partkey", "integer"), ("p_name", "string"), ("p_mfgr", "string"), ("p_brand", "string"),
             ("p_type", "string"), ("p_size", "integer"), ("p_container", "string"), ("p_retailprice", "double"),
             ("p_comment", "string")],
    "supplier": [("s_suppkey", "integer"), ("s_name", "string"), ("s_address", "string"), ("s_nationkey", "integer"),
                 ("s_phone", "string"), ("s_acctbal", "double"), ("s_comment", "string")],
    "customer": [("c_custkey", "integer"), ("c_name", "string"), ("c_address", "string"), ("c_nationkey", "integer"),
                 ("c_phone", "string"), ("c_acctbal", "double"), ("c_mktsegment", "string"), ("c_comment", "string")],
    "custnation": [("cn_nationkey", "integer"), ("cn_name", "string"), ("cn_regionkey", "integer"),
                   ("cn_comment", "string")],
    "custregion": [("cr_regionkey", "integer"), ("cr_name", "string"), ("cr_comment", "string")],
    "suppnation": [("sn_nationkey", "integer"), ("sn_name", "string"), ("sn_regionkey", "integer"),
                   ("sn_comment", "string")],
    "suppregion": [("sr_regionkey", "integer"), ("sr_name", "string"), ("sr_comment", "string")],
}


def star_tables(df):
    """Split the flattened table back into the star-schema tables (distinct rows per key)."""
    import pandas as pd

    nat_key = {n: i for i, (n, _) in enumerate(NATIONS)}
    nat_reg = {n: r for n, r in NATIONS}
    out = {}
    li = df.rename(columns={"o_orderkey": "l_orderkey"})
    out["lineitembase"] = li[[c for c, _ in STAR_SCHEMAS["lineitembase"]]].reset_index(drop=True)
    out["orders"] = df[[c for c, _ in STAR_SCHEMAS["orders"]]].drop_duplicates("o_orderkey").reset_index(drop=True)
    out["partsupp"] = df[[c for c, _ in STAR_SCHEMAS["partsupp"]]].drop_duplicates(
        ["ps_partkey", "ps_suppkey"]).reset_index(drop=True)
    p = df[["l_partkey"] + [c for c, _ in STAR_SCHEMAS["part"][1:]]].rename(columns={"l_partkey": "p_partkey"})
    out["part"] = p.drop_duplicates("p_partkey").reset_index(drop=True)
    s = df[["l_suppkey", "s_name", "s_address", "s_nation", "s_phone", "s_acctbal", "s_comment"]].drop_duplicates(
        "l_suppkey")
    out["supplier"] = pd.DataFrame({"s_suppkey": s.l_suppkey, "s_name": s.s_name, "s_address": s.s_address,
                                    "s_nationkey": s.s_nation.map(nat_key), "s_phone": s.s_phone,
                                    "s_acctbal": s.s_acctbal, "s_comment": s.s_comment}).reset_index(drop=True)
    c = df[["o_custkey", "c_name", "c_address", "c_nation", "c_phone", "c_acctbal", "c_mktsegment",
            "c_comment"]].drop_duplicates("o_custkey")
    out["customer"] = pd.DataFrame({"c_custkey": c.o_custkey, "c_name": c.c_name, "c_address": c.c_address,
                                    "c_nationkey": c.c_nation.map(nat_key), "c_phone": c.c_phone,
                                    "c_acctbal": c.c_acctbal, "c_mktsegment": c.c_mktsegment,
                                    "c_comment": c.c_comment}).reset_index(drop=True)
    nations = pd.DataFrame({"k": [nat_key[n] for n, _ in NATIONS], "n": [n for n, _ in NATIONS],
                            "r": [nat_reg[n] for n, _ in NATIONS], "c": [f"nation {n}" for n, _ in NATIONS]})
    regions = pd.DataFrame({"k": list(range(len(REGIONS))), "n": REGIONS, "c": [f"region {r}" for r in REGIONS]})
    for pre in ("cn", "sn"):
        out[f"{pre[0]}{'ustnation' if pre == 'cn' else 'uppnation'}"] = nations.rename(
            columns={"k": f"{pre}_nationkey", "n": f"{pre}_name", "r": f"{pre}_regionkey", "c": f"{pre}_comment"})
    for pre in ("cr", "sr"):
        out[f"{pre[0]}{'ustregion' if pre == 'cr' else 'uppregion'}"] = regions.rename(
            columns={"k": f"{pre}_regionkey", "n": f"{pre}_name", "c": f"{pre}_comment"})
    return out


def star_ddl(datasource: str = "tpch", fact_db: str = "default", dim_db: str = "default",
             table: str = "lineitem", extra_options: str = "", column_mapping: Optional[dict] = None) -> str:
    """Star-schema fact table DDL (``tc/StarSchemaBaseTest.scala:88-101``); ``table`` renames the fact
    table (``SelectQueryTest.scala:51-63`` registers ``lineitem_select`` over the same index)."""
    import json

    ss = star_schema_json(fact_db, dim_db)
    if table != "lineitem":
        ss = ss.replace(f"{fact_db}.lineitem\"", f"{fact_db}.{table}\"")
    return (f"CREATE TABLE if not exists {fact_db}.{table} USING org.sparklinedata.druid OPTIONS ("
            f"sourceDataframe \"{fact_db}.lineitembase\", timeDimensionColumn \"l_shipdate\", "
            f"druidDatasource \"{datasource}\", druidHost 'localhost', "
            f"columnMapping '{json.dumps(COLUMN_MAPPING if column_mapping is None else column_mapping)}', "
            f"numProcessingThreadsPerHistorical '1', "
            f"functionalDependencies '{json.dumps(FUNCTIONAL_DEPENDENCIES)}', "
            f"starSchema '{ss}'{extra_options})")
