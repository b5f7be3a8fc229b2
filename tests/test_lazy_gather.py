"""Deferred row gathers of the SQL executor (sql/execute.py LazyGather): a gather runs only when
its column is read, composed gathers give the eager answer, and a statement's result holds real
columns."""
import numpy as np
import pandas as pd

from spark_druid_olap_amd.sql import ast as A
from spark_druid_olap_amd.sql.execute import Batch, LazyGather, LazySeries, lazy_series


def _batch():
    refs = [A.Ref(1, "a", "bigint"), A.Ref(2, "b", "double"), A.Ref(3, "c", "string")]
    cols = {1: lazy_series(np.arange(10, dtype=np.int64)), 2: pd.Series(np.arange(10) * 0.5),
            3: pd.Series([f"s{i}" for i in range(10)])}
    return Batch(refs, cols, 10)


def test_take_defers_until_read_and_composes():
    b = _batch()
    t = b.take(np.array([9, 7, 5, 3, 1]))
    assert all(type(dict.__getitem__(t.cols, k)) is LazyGather for k in t.cols)
    u = t.take(np.array([4, 0]))  # gather of a gather
    assert list(u.cols[1]) == [1, 9] and list(u.cols[2]) == [0.5, 4.5] and list(u.cols[3]) == ["s1", "s9"]
    assert type(dict.__getitem__(u.cols, 1)) is not LazyGather  # read -> memoized as a Series
    assert type(dict.__getitem__(u.cols, 3)) is not LazyGather
    assert list(u.cols.array(2)) == [0.5, 4.5]


def test_unread_columns_are_never_gathered():
    calls = []

    def make():
        calls.append(1)
        return pd.Series(np.arange(10))

    refs = [A.Ref(1, "a", "bigint"), A.Ref(2, "b", "bigint")]
    b = Batch(refs, {1: LazySeries(make), 2: pd.Series(np.arange(10))}, 10)
    t = b.take(np.array([1, 2]))
    assert list(t.cols[2]) == [1, 2] and not calls  # column 1 never built, never gathered
    t.materialize_gathers()
    assert calls == [1] and list(t.cols[1]) == [1, 2]
