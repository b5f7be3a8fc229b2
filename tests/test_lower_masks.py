"""Dictionary-id mask helpers of the lowering (engine/lower.py): packed F_IN_SET words, run counts
and the identity cache that lets every parameterization of a LIKE template reuse one mask's
statistics."""
import numpy as np
import pytest

from spark_druid_olap_amd.engine import lower as L


def _pack_ref(mask):
    words = np.zeros((len(mask) + 63) // 64, dtype=np.uint64)
    for i in np.flatnonzero(mask):
        words[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
    return words.view(np.int64)


def _runs_ref(mask):
    out, start = [], None
    for i, v in enumerate(mask):
        if v and start is None:
            start = i
        if not v and start is not None:
            out.append((start, i))
            start = None
    if start is not None:
        out.append((start, len(mask)))
    return out


@pytest.mark.parametrize("n", [1, 7, 64, 65, 200, 1000])
@pytest.mark.parametrize("p", [0.0, 0.03, 0.5, 0.97, 1.0])
def test_pack_and_runs_match_reference(n, p):
    m = np.random.default_rng(n).random(n) < p
    assert (L.pack_bitset(m) == _pack_ref(m)).all()
    st = L.MaskStats(m)
    assert st.k == int(m.sum())
    assert L._runs(m) == _runs_ref(m)
    assert st.runs == len(_runs_ref(m))
    assert st.neg_runs == len(_runs_ref(~m))
    if st.k:
        nz = np.flatnonzero(m)
        assert (st.lo, st.hi) == (nz[0], nz[-1] + 1)


def test_runs_limit_skips_listing():
    m = np.zeros(1000, dtype=bool)
    m[::2] = True  # 500 runs
    assert L._runs(m, limit=10) is None
    assert len(L._runs(m, limit=500)) == 500


def test_mask_stats_cached_by_identity():
    m = np.zeros(L._MASK_STATS_MIN + 5, dtype=bool)
    m[10:20] = True
    a = L.mask_stats(m)
    assert L.mask_stats(m) is a
    other = m.copy()
    assert L.mask_stats(other) is not a          # an equal but different array is its own entry
    small = np.ones(8, dtype=bool)
    assert L.mask_stats(small) is not L.mask_stats(small)  # small masks are not cached

