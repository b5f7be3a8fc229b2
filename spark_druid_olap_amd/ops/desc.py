"""Byte-exact mirror of ``ops/csrc/scan_desc.h`` as numpy structured dtypes.

The host lowers a query into a ``ScanProgram`` (engine/lower.py), ``pack()`` turns it into the
C struct bytes, and the bytes are copied once to device memory; the kernel reads them with
scalar loads.  ``tests/test_native_layout.py`` checks these sizes/offsets against the compiled
extension's ``layout()``.
"""
from __future__ import annotations

import numpy as np

MAX_COLS = 24
MAX_FOPS = 48
MAX_KOPS = 8
MAX_AOPS = 12
MAX_EOPS = 64
MAX_ZONES = 4
MAX_RANGES = 8
MAX_SLOTS = 16
MAX_BM = 8
PAYLOAD_BASE = 8
STACK_DEPTH = 6
CHUNK_ROWS = 4096
CHUNK_WORDS = CHUNK_ROWS // 64

# opcodes
F_TRUE, F_BITMAP, F_ID_RANGE, F_IN_SET, F_INT_RANGE, F_FLT_RANGE, F_AND, F_OR, F_NOT, F_FALSE, F_BITMAP_OR, \
    F_EXPR = range(12)
K_ID, K_REMAP, K_TIME, K_INT = range(4)
A_COUNT, A_SUM_I, A_SUM_F, A_MIN_I, A_MAX_I, A_MIN_F, A_MAX_F, A_HLL, A_SUM_X, A_HLL_STORED, A_ROWID, \
    A_HLL_CODE, A_THETA = range(13)  # (A_THETA: a theta producer's 62-bit KMV hash of a column, JIT only)
HLL_KINDS = (A_HLL, A_HLL_CODE)  # query-time HLL over a column (hashed per row / precomputed code)
S_SUM_I, S_SUM_F, S_MIN_I, S_MAX_I = range(4)
E_COL, E_CONST, E_ADD, E_SUB, E_MUL, E_DIV, E_NEG, E_ABS, E_MIN, E_MAX = range(10)
E_FLOOR, E_CEIL, E_SQRT, E_LOG, E_EXP, E_MOD, E_PMOD, E_POW, E_LUT = range(10, 19)
E_UNARY = (E_NEG, E_ABS, E_FLOOR, E_CEIL, E_SQRT, E_LOG, E_EXP)
M_DENSE_LDS, M_DENSE_GLOBAL, M_HASH, M_MASK, M_PART = range(5)

INT64_MAX = np.iinfo(np.int64).max
INT64_MIN = np.iinfo(np.int64).min

COLREF = np.dtype([("ptr", "<u8"), ("dtype", "<i4"), ("meta", "<i4")], align=True)
FOP = np.dtype([("op", "<i4"), ("col", "<i4"), ("flags", "<i4"), ("pad", "<i4"), ("lo", "<i8"), ("hi", "<i8"),
                ("flo", "<f8"), ("fhi", "<f8"), ("bits", "<u8")], align=True)
KOP = np.dtype([("kind", "<i4"), ("col", "<i4"), ("tfield", "<i4"), ("pad", "<i4"), ("stride", "<i8"),
                ("base", "<i8"), ("card", "<i8"), ("unit_ms", "<i8"), ("tz_ms", "<i8"), ("period_ms", "<i8"),
                ("origin_ms", "<i8"), ("remap", "<u8")], align=True)
AOP = np.dtype([("kind", "<i4"), ("col", "<i4"), ("expr_off", "<i4"), ("expr_len", "<i4"), ("filt_off", "<i4"),
                ("filt_len", "<i4"), ("slot", "<i4"), ("hll_lds_off", "<i4"), ("hll_regs", "<u8"),
                ("salt", "<i8"), ("sk_off", "<u8"), ("sk_val", "<u8")], align=True)
EOP = np.dtype([("op", "<i4"), ("col", "<i4"), ("c", "<f8")], align=True)
ZONEP = np.dtype([("col", "<i4"), ("pad", "<i4"), ("lo", "<i8"), ("hi", "<i8"), ("zmin", "<u8"), ("zmax", "<u8")],
                 align=True)
RANGE = np.dtype([("lo", "<i8"), ("hi", "<i8"), ("chunk_begin", "<i8"), ("nchunks", "<i8")], align=True)

SCANDESC = np.dtype([
    ("ncols", "<i4"), ("nfops", "<i4"), ("nkops", "<i4"), ("naggs", "<i4"),
    ("neops", "<i4"), ("nranges", "<i4"), ("nzones", "<i4"), ("nslots", "<i4"),
    ("mode", "<i4"), ("dedup", "<i4"), ("hll_lds", "<i4"), ("hll_p", "<i4"),
    ("nhll", "<i4"), ("lds_bytes", "<i4"), ("filter_len", "<i4"), ("pad0", "<i4"),
    ("G", "<i8"), ("total_chunks", "<i8"), ("num_rows", "<i8"),
    ("out_acc", "<u8"), ("out_keys", "<u8"), ("hash_cap", "<i8"), ("overflow", "<u8"),
    ("out_mask", "<u8"), ("out_count", "<u8"),
    ("slot_init", "<i8", (MAX_SLOTS,)), ("slot_op", "<i4", (MAX_SLOTS,)),
    ("cols", COLREF, (MAX_COLS,)), ("fops", FOP, (MAX_FOPS,)), ("kops", KOP, (MAX_KOPS,)),
    ("aops", AOP, (MAX_AOPS,)), ("eops", EOP, (MAX_EOPS,)), ("zones", ZONEP, (MAX_ZONES,)),
    ("ranges", RANGE, (MAX_RANGES,)),
    ("nfc", "<i4"), ("npc", "<i4"), ("pre_off", "<i4"), ("pre_len", "<i4"), ("final_pre", "<i4"), ("nbm", "<i4"),
    ("nplanes", "<i4"), ("lds_cache_off", "<i4"), ("lds_wave_bytes", "<i4"), ("unroll", "<i4"),
    ("narrow4", "<i4"), ("pad2", "<i4"),
    ("bm_bits", "<u8", (MAX_BM,)), ("bm_stride", "<i8", (MAX_BM,)), ("bm_count", "<i8", (MAX_BM,)),
    ("part_recs", "<u8"), ("part_counts", "<u8"), ("part_base", "<u8"), ("part_shift", "<i4"), ("part_n", "<i4"),
], align=True)


def layout() -> dict:
    d = {"ScanDesc": SCANDESC.itemsize, "ColRef": COLREF.itemsize, "FOp": FOP.itemsize, "KOp": KOP.itemsize,
         "AOp": AOP.itemsize, "EOp": EOP.itemsize, "ZoneP": ZONEP.itemsize, "Range": RANGE.itemsize}
    for f in ("cols", "fops", "kops", "aops", "eops", "zones", "ranges", "slot_init"):
        d["off_" + f] = SCANDESC.fields[f][1]
    return d


def new_desc() -> np.ndarray:
    return np.zeros(1, dtype=SCANDESC)
