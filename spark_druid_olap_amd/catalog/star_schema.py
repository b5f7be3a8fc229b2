"""Star schema model: which dimension tables join to the fact table, along which keys.

Parity: ``sd/metadata/StarSchemaInfo.scala`` -- ``StarSchemaInfo`` JSON (34-86), ``StarSchema``
(172-296: ``getUniqueTable``, ``isStarJoin`` 215-275, ``isJoiningColumn``), the builder with its
validation errors (354-463: n-1/1-1 relations only, unique join path to every table, column names
unique across the schema, every declared table reachable).  Used by the join-elimination rewrite:
an inner equi-join tree over these tables collapses onto the single denormalized index.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Set, Tuple

MANY_TO_ONE = "n-1"
ONE_TO_ONE = "1-1"


class StarSchemaError(ValueError):
    pass


@dataclass
class StarRelationInfo:
    leftTable: str
    rightTable: str
    relationType: str
    joinCondition: List[Tuple[str, str]]


@dataclass
class StarSchemaInfo:
    factTable: str
    relations: List[StarRelationInfo] = field(default_factory=list)

    @staticmethod
    def parse(s) -> "StarSchemaInfo":
        d = json.loads(s) if isinstance(s, str) else s
        rels = []
        for r in d.get("relations", []):
            rt = r.get("relationType", MANY_TO_ONE)
            if rt not in (MANY_TO_ONE, ONE_TO_ONE):
                raise StarSchemaError(f"unsupported relationType {rt}")
            jc = [(c["leftAttribute"], c["rightAttribute"]) for c in r.get("joinCondition", [])]
            rels.append(StarRelationInfo(r["leftTable"], r["rightTable"], rt, jc))
        return StarSchemaInfo(d["factTable"], rels)

    def to_json(self) -> dict:
        return {"factTable": self.factTable,
                "relations": [{"leftTable": r.leftTable, "rightTable": r.rightTable, "relationType": r.relationType,
                               "joinCondition": [{"leftAttribute": a, "rightAttribute": b} for a, b in r.joinCondition]}
                              for r in self.relations]}


@dataclass
class StarTable:
    name: str
    parent: Optional[str] = None                     # table this one joins up to
    relation_type: Optional[str] = None
    joining_keys: Set[Tuple[str, str]] = field(default_factory=set)  # (this table col, parent col)

    def is_joining_column(self, table: Optional[str], column: str) -> bool:
        if table is not None and table.lower() != _short(self.name):
            return False
        return any(column.lower() == a.lower() for a, _ in self.joining_keys)


def _short(name: str) -> str:
    return name.split(".")[-1].lower()


class StarSchema:
    UNKNOWN = "<unknownTable>"

    def __init__(self, info: StarSchemaInfo, fact: StarTable, table_map: Dict[str, StarTable],
                 attr_map: Dict[str, StarTable]):
        self.info = info
        self.fact = fact
        self.table_map = table_map      # short lower name -> StarTable
        self.attr_map = attr_map        # lower column name -> StarTable

    @property
    def is_flat(self) -> bool:
        return len(self.table_map) == 1

    def table_of(self, column: str) -> Optional[StarTable]:
        return self.attr_map.get(column.lower())

    def unique_table(self, cols: Sequence[str]) -> Optional[str]:
        ts = {(self.attr_map[c.lower()].name if c.lower() in self.attr_map else self.UNKNOWN) for c in cols}
        if len(ts) == 1 and self.UNKNOWN not in ts:
            return _short(next(iter(ts)))
        return None

    def is_star_join(self, left_cols: Sequence[str], right_cols: Sequence[str]) -> Optional[Tuple[str, str]]:
        lt = self.unique_table(left_cols)
        rt = self.unique_table(right_cols)
        if lt is None or rt is None:
            return None
        L, R = self.table_map[lt], self.table_map[rt]
        flip = False
        if L.parent is not None and _short(L.parent) == rt:
            cond = L.joining_keys
        elif R.parent is not None and _short(R.parent) == lt:
            cond = R.joining_keys
            flip = True
        else:
            return None
        lk, rk = (right_cols, left_cols) if flip else (left_cols, right_cols)
        keys = {(a.lower(), b.lower()) for a, b in zip(lk, rk)}
        want = {(a.lower(), b.lower()) for a, b in cond}
        if keys == want:
            return (lt, rt)
        return None

    def is_joining_column(self, table: Optional[str], column: str) -> bool:
        return any(t.is_joining_column(table, column) for t in self.table_map.values())

    def pretty(self) -> str:
        lines = [f"FactTable={self.fact.name}"]
        for k, t in self.table_map.items():
            lines.append(f"{k} -> parent={t.parent} keys={sorted(t.joining_keys)}")
        return "\n".join(lines)

    # --------------------------------------------------------------------------------- builder
    @staticmethod
    def build(source_name: str, info: StarSchemaInfo, columns_of: Callable[[str], List[str]]) -> "StarSchema":
        graph: Dict[str, Dict[str, Tuple[str, Set[Tuple[str, str]]]]] = {}
        errors = []
        for r in info.relations:
            lrs = graph.setdefault(_short(r.leftTable), {})
            if _short(r.rightTable) in lrs:
                errors.append(f"multiple join conditions for '{r.leftTable}' and '{r.rightTable}'")
                continue
            lrs[_short(r.rightTable)] = (r.relationType, {(a, b) for a, b in r.joinCondition})
            if r.relationType == ONE_TO_ONE:
                graph.setdefault(_short(r.rightTable), {})[_short(r.leftTable)] = (
                    r.relationType, {(b, a) for a, b in r.joinCondition})
        if errors:
            raise StarSchemaError("\n".join(errors))
        table_map: Dict[str, StarTable] = {}
        attr_map: Dict[str, StarTable] = {}
        traversed: Set[Tuple[str, str]] = set()

        def add_columns(tab: str, st: StarTable):
            for c in columns_of(tab):
                if c.lower() in attr_map:
                    raise StarSchemaError(f"Column {c} is not unique across Star Schema; in tables "
                                          f"{attr_map[c.lower()].name}, {tab}")
                attr_map[c.lower()] = st

        fact = StarTable(_short(info.factTable))
        table_map[fact.name] = fact
        add_columns(source_name, fact)
        frontier = [fact.name]
        while frontier:
            nxt = []
            for t in frontier:
                for child, (rt, jc) in graph.get(t, {}).items():
                    if child in table_map:
                        if (child, t) not in traversed and (t, child) not in traversed:
                            raise StarSchemaError(f"multiple join paths to table '{child}'")
                        continue
                    traversed.add((t, child))
                    st = StarTable(child, t, rt, {(b, a) for a, b in jc})
                    table_map[child] = st
                    add_columns(child, st)
                    nxt.append(child)
            frontier = nxt
        missing = []
        for r in info.relations:
            for t in (r.leftTable, r.rightTable):
                if _short(t) not in table_map:
                    missing.append(f"Table '{t}' is not part of the join Graph")
        if missing:
            raise StarSchemaError("\n".join(sorted(set(missing))))
        return StarSchema(info, fact, table_map, attr_map)
