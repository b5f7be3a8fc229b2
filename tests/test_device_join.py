"""Host equi-join of aggregated Druid results (sql/execute.py _numeric_key_join): the GPU variant
must return exactly the numpy variant's (left row, right row) pairs, in the same order."""
import numpy as np
import pandas as pd
import pytest

from spark_druid_olap_amd.sql import execute as X


def _case(n_l, n_r, seed, multi=False, flt=False):
    rng = np.random.default_rng(seed)
    lk = [pd.Series(rng.integers(0, n_r // 2, n_l))]
    rk = [pd.Series(rng.integers(0, n_r // 2, n_r))]
    if multi:
        lk.append(pd.Series(rng.integers(0, 3, n_l)))
        rk.append(pd.Series(rng.integers(0, 3, n_r)))
    if flt:
        lk[0] = lk[0].astype(np.float64)
    lok = rng.random(n_l) > 0.05
    rok = rng.random(n_r) > 0.05
    return lk, rk, lok, rok


def test_host_join_matches_pandas_merge():
    lk, rk, lok, rok = _case(3000, 800, 1, multi=True)
    li, ri = X._numeric_key_join(lk, rk, lok, rok)
    l = pd.DataFrame({"a": lk[0], "b": lk[1], "li": np.arange(3000)})[lok]
    r = pd.DataFrame({"a": rk[0], "b": rk[1], "ri": np.arange(800)})[rok]
    m = l.merge(r, on=["a", "b"], how="inner")
    assert sorted(zip(li.tolist(), ri.tolist())) == sorted(zip(m.li.tolist(), m.ri.tolist()))
    assert (np.diff(li) >= 0).all()  # left-row order


@pytest.mark.gpu
@pytest.mark.parametrize("multi,flt", [(False, False), (True, False), (False, True)])
def test_device_join_equals_host(multi, flt, monkeypatch):
    lk, rk, lok, rok = _case(400_000, 60_000, 7, multi, flt)
    monkeypatch.setattr(X, "_DEVICE_JOIN_MIN", 1 << 62)
    host = X._numeric_key_join(lk, rk, lok, rok)
    monkeypatch.setattr(X, "_DEVICE_JOIN_MIN", 1)
    dev = X._numeric_key_join(lk, rk, lok, rok)
    assert np.array_equal(host[0], dev[0]) and np.array_equal(host[1], dev[1])


@pytest.mark.gpu
def test_direct_address_join_for_unique_right_keys(monkeypatch):
    """Unique integer right keys (a group-by result joined on its key, TPC-H Q17) take the
    direct-address path: same pairs, same order as the host join."""
    rng = np.random.default_rng(11)
    rkeys = rng.permutation(2_000_000)[:20_000] + 5
    lk = [pd.Series(rng.choice(np.concatenate([rkeys, rng.integers(0, 3_000_000, 5_000)]), 450_000))]
    rk = [pd.Series(rkeys)]
    lok = rng.random(450_000) > 0.02
    rok = rng.random(20_000) > 0.02
    calls = []
    real = X._unique_right_join_device
    monkeypatch.setattr(X, "_unique_right_join_device", lambda *a: calls.append(1) or real(*a))
    monkeypatch.setattr(X, "_DEVICE_JOIN_MIN", 1 << 62)
    host = X._numeric_key_join(lk, rk, lok, rok)
    monkeypatch.setattr(X, "_DEVICE_JOIN_MIN", 1)
    dev = X._numeric_key_join(lk, rk, lok, rok)
    assert calls and np.array_equal(host[0], dev[0]) and np.array_equal(host[1], dev[1])
