"""Late-materialized result columns.

Group-by results over dictionary-encoded dimensions come back from the GPU as dictionary ids.
``DictColumn`` keeps them encoded (codes + the dimension's sorted dictionary, the layout of an
Arrow DictionaryArray / pandas Categorical) and decodes to Python values only when a consumer
actually reads them (``rows()``, ``to_pandas()``, a Thrift fetch page).  A 1.2M-group TPC-H Q3
result therefore costs one small D2H copy of int codes instead of 1.2M Python string objects.
"""
from __future__ import annotations

from typing import Any, Iterator

import numpy as np


class DictColumn:
    """Dictionary-encoded column: values = dictionary.decode(codes)."""

    __array_priority__ = 10

    def __init__(self, codes: np.ndarray, dictionary):
        codes = np.asarray(codes)
        self.codes = codes if codes.dtype in (np.int16, np.int32, np.int64) else codes.astype(np.int64)
        self.dictionary = dictionary
        self._decoded = None

    @property
    def dtype(self):
        return np.dtype(object)

    @property
    def shape(self):
        return self.codes.shape

    def __len__(self) -> int:
        return len(self.codes)

    def to_numpy(self) -> np.ndarray:
        if self._decoded is None:
            self._decoded = np.asarray(self.dictionary.decode(self.codes), dtype=object)
        return self._decoded

    def __array__(self, dtype=None, copy=None):
        a = self.to_numpy()
        return a.astype(dtype) if dtype is not None else a

    def take(self, idx) -> "DictColumn":
        return DictColumn(self.codes[idx], self.dictionary)

    def __getitem__(self, i):
        if isinstance(i, (int, np.integer)):
            return self.dictionary.value(int(self.codes[i]))
        return self.take(i)

    def __iter__(self) -> Iterator[Any]:
        return iter(self.to_numpy().tolist())

    def tolist(self):
        return self.to_numpy().tolist()

    def __repr__(self) -> str:
        return f"DictColumn(n={len(self)}, card={len(self.dictionary)})"


def take(col, idx):
    """Index a result column without forcing dictionary decoding."""
    if isinstance(col, DictColumn):
        return col.take(idx)
    return np.asarray(col)[idx]


def materialize(col) -> np.ndarray:
    return col.to_numpy() if isinstance(col, DictColumn) else np.asarray(col)
