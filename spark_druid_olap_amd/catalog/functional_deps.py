"""Functional dependencies between dimensions and the group-by cardinality estimate.

Parity: ``sd/metadata/FunctionalDependency.scala`` -- ``FunctionalDependency`` (27-29),
``DependencyGraph`` with a transitive closure (141-190) and ``estimateCardinality`` (59-83): the
cardinality of a GROUP BY is the product of dimension cardinalities after dropping every dimension
functionally determined by another grouped dimension.  The GPU planner uses the estimate to pick
dense-LDS vs hash group-by tables and to size hash tables.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Callable, Dict, List, Sequence

ONE_TO_ONE = "1-1"
MANY_TO_ONE = "n-1"


@dataclass
class FunctionalDependency:
    col1: str
    col2: str
    type: str

    @staticmethod
    def parse_list(s) -> List["FunctionalDependency"]:
        d = json.loads(s) if isinstance(s, str) else (s or [])
        out = []
        for x in d:
            t = x.get("type", MANY_TO_ONE)
            if t not in (ONE_TO_ONE, MANY_TO_ONE):
                raise ValueError(f"unsupported functional dependency type {t}")
            out.append(FunctionalDependency(x["col1"], x["col2"], t))
        return out


class DependencyGraph:
    """closure[a][b] == True iff a functionally determines b (a -> b), transitively."""

    def __init__(self, dims: Sequence[str], fds: Sequence[FunctionalDependency]):
        self.dims = list(dims)
        idx = {d: i for i, d in enumerate(self.dims)}
        n = len(self.dims)
        m = [[i == j for j in range(n)] for i in range(n)]
        for fd in fds:
            if fd.col1 not in idx or fd.col2 not in idx:
                continue
            a, b = idx[fd.col1], idx[fd.col2]
            m[a][b] = True
            if fd.type == ONE_TO_ONE:
                m[b][a] = True
        # Floyd-Warshall style closure (FunctionalDependency.scala:176-184)
        for k in range(n):
            mk = m[k]
            for i in range(n):
                if m[i][k]:
                    mi = m[i]
                    for j in range(n):
                        if mk[j]:
                            mi[j] = True
        self.idx = idx
        self.m = m

    def determines(self, a: str, b: str) -> bool:
        if a not in self.idx or b not in self.idx:
            return a == b
        return self.m[self.idx[a]][self.idx[b]]

    def estimate_cardinality(self, dims: Sequence[str], card: Callable[[str], int]) -> int:
        dims = list(dict.fromkeys(dims))
        keep = []
        for d in dims:
            dominated = any(o != d and self.determines(o, d) and not (self.determines(d, o) and dims.index(o) > dims.index(d))
                            for o in dims)
            if not dominated:
                keep.append(d)
        out = 1
        for d in keep:
            out *= max(int(card(d)), 1)
        return out
