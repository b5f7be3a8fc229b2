"""Per-query kernel specialization (JIT) for the fused scan.

The precompiled interpreter (``csrc/olap_scan.hip``) decodes opcodes, column widths and key
strides from the descriptor at run time; on CDNA4 that costs ~80 scalar instructions and several
dependent scalar loads per LDS-DMA (measured: profiles/pmc_shipdate_sf10_v3.txt).  Here the same
ScanProgram is emitted as C++ in which every opcode, column width, LDS plane, key stride and
aggregator is a compile-time constant and filters are straight boolean expressions over
``__ballot`` masks / bitmap words; hipRTC compiles it for gfx950 once per query shape and the
code object is cached on disk by source hash.  Device pointers still come from the descriptor,
so one compiled kernel serves every shard/rank and every re-execution of a prepared query.
"""
from __future__ import annotations

import hashlib
import os
import threading
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch

from . import desc as D

CSRC = Path(__file__).resolve().parent / "csrc"
OPTS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics", f"-I{CSRC}"]
W = 8  # waves per block (512 threads)

_lock = threading.Lock()
_handles: Dict[str, int] = {}


def cache_dir() -> Path:
    p = Path(os.environ.get("SDO_JIT_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "sdo_jit")))
    p.mkdir(parents=True, exist_ok=True)
    return p


@dataclass
class ColInfo:
    name: str
    idx: int       # descriptor column index
    lg: int
    sgn: bool
    flt: bool
    plane: int     # LDS staging plane (-1: bit-packed, always loaded into registers)
    pw: int = 0    # bit-packed width (segment/packed.py); 0 = plain column
    pbase: int = 0


@dataclass
class JitLayout:
    acc_off: int
    acc_bytes: int
    hll_off: int
    hll_bytes: int
    cache_off: int
    wave_bytes: int
    total: int
    ncopy: int
    regstage: bool = False
    shared: bool = False  # one accumulator copy per workgroup (LDS atomics shared by its 8 waves)
    G: int = 0  # groups the LDS table is sized for (a size class >= the program's G)


def col_infos(prog) -> Dict[int, ColInfo]:
    from ..engine.lower import column_tensor

    out = {}
    plane = 0
    packed = getattr(prog, "packed", None) or {}
    for base, names in ((0, prog.fcols), (D.PAYLOAD_BASE, prog.pcols)):
        for j, name in enumerate(names):
            t = column_tensor(prog.ds, name)
            lg = {1: 0, 2: 1, 4: 2, 8: 3}[t.element_size()]
            pk = packed.get(name)
            if pk is not None:
                out[base + j] = ColInfo(name, base + j, lg, False, False, -1, pk.width, pk.base)
                continue
            out[base + j] = ColInfo(name, base + j, lg, t.dtype in (torch.int16, torch.int32, torch.int64),
                                    t.dtype.is_floating_point, plane)
            plane += 2 if lg == 3 else 1
    return out


JIT_LITERALS = False  # (tools: literal-specialized shape kernels from the first compile)
PART_MAX_BUCKETS = 1024  # level-1 buckets of the partitioned group-by (split kernel LDS cursors)
PART_HIST_BYTES = 4 * PART_MAX_BUCKETS  # (sdo_device.h PART_HIST_BUCKETS counters)


def part_positions(nch: int, grid: int):
    """(number of positions, position of every chunk) in producer-workgroup order: the M_PART
    producer deals chunk c to wave c mod (grid x W), and block b's waves own the positions
    [b x S, (b + 1) x S) with S = ceil(nch / (grid x W)) x W -- chunk j x grid x W + b x W + v at
    b x S + j x W + v, the unused ones empty.  The level-1 split with grid blocks over the positions
    then gives block b exactly producer block b's records: the slice its histogram counted."""
    import numpy as np

    TW = grid * W
    per = -(-nch // TW) * W
    c = np.arange(nch, dtype=np.int64)
    gw = c % TW
    pos = (gw // W) * per + (c // TW) * W + gw % W
    return grid * per, pos


def part_fields(prog, cols=None) -> List[Tuple[int, int]]:
    """(slot, u32 words) of every aggregator's value in a partition record (partition.hip
    part_agg_kernel): 0 = an unfiltered count (implicit 1), 1 = a value that fits int32 (filtered
    counts, integer columns of <= 4 signed / <= 2 unsigned bytes), 2 = int64 / double bits."""
    if not hasattr(prog, "aops"):  # planner-level estimate without a lowered program: int64 values
        return [(s, 2) for s in range(max(1, prog.nslots))]
    cols = col_infos(prog) if cols is None else cols
    out = []
    for a in prog.aops:
        kind = a["kind"]
        if kind in (D.A_HLL, D.A_HLL_CODE, D.A_HLL_STORED):
            continue
        if kind == D.A_COUNT:
            out.append((a["slot"], 1 if a.get("filt_len") else 0))
            continue
        if kind == D.A_ROWID:
            out.append((a["slot"], 1))  # u32 row id (emit producers, engine/device_exec.py PreparedEmit)
            continue
        if kind == D.A_THETA:
            out.append((a["slot"], 2))  # 62-bit KMV hash (theta producers, engine/device_exec.py PreparedTheta)
            continue
        w = 2
        if kind in (D.A_SUM_I, D.A_MIN_I, D.A_MAX_I) and not a.get("expr") and a.get("col") in cols:
            c = cols[a["col"]]
            if not c.flt and not c.pw and (c.lg <= 1 or (c.lg == 2 and c.sgn)):
                w = 1
        out.append((a["slot"], w))
    return out


FORCE_HASHED = False  # tests: the hashed layout for any key space


def part_hashed(prog) -> bool:
    """Key spaces beyond 32 bits partition by a 32-bit hash of the 64-bit key and aggregate sparsely
    (ops/csrc/partition.hip part_hash_agg_kernel): records are (hash, key lo, key hi, values...)."""
    return prog.G >= (1 << 32) or FORCE_HASHED


def part_record_words(prog) -> int:
    """Header words of a partition record: the u32 key, or hash + 64-bit key."""
    return 3 if part_hashed(prog) else 1


PART_HLL = True  # HLL aggregators ride the partitioned records as (bucket << 8 | rho) words
PART_HLL_MAX_BYTES = 1 << 30  # register tables ([G][2^p] bytes per HLL) the partitioned path writes


def part_stored_count(prog) -> int:
    """Stored (rolled-up hyperUnique) sketches a partition record carries: one row-id word each,
    after the query-time HLL words (partition.hip part_agg_kernel unions the row's stored pairs)."""
    if not hasattr(prog, "aops"):
        return len(getattr(prog, "stored_hll", None) or [])
    return sum(1 for a in prog.aops if a["kind"] == D.A_HLL_STORED)


def part_hll_count(prog) -> int:
    """HLL register tables of a partitioned group-by: query-time HLL words plus stored-sketch row
    words (one word each per record, after the value fields; the query-time ones first)."""
    if not hasattr(prog, "aops"):
        return int(prog.nhll) + part_stored_count(prog)
    return sum(1 for a in prog.aops if a["kind"] in D.HLL_KINDS) + part_stored_count(prog)


def part_eligible(prog) -> bool:
    """The partitioned group-by handles every slot operator and any key space (beyond 32 bits by
    hash), and query-time HLL sketches -- plus stored (rolled-up) sketches on dense (u32) key
    spaces -- whose register tables fit PART_HLL_MAX_BYTES."""
    slots = getattr(prog, "slots", None)
    n = len(slots) if slots is not None else prog.nslots
    if not (n > 0 and 0 < prog.G < (1 << 62) and not prog.empty):
        return False
    nst = len(getattr(prog, "stored_hll", None) or [])
    if nst and int(getattr(getattr(prog, "ds", None), "num_rows", 0)) >= 0xFFFFFFFF:
        return False  # (a stored sketch's record word is the u32 row id; all-ones = filtered out)
    if prog.nhll or nst:
        nh = part_hll_count(prog)
        if not (PART_HLL and nh == prog.nhll + nst and nh <= 4):
            return False
        if part_hashed(prog):
            if nst:  # (the hashed sparse aggregation has no stored-sketch union)
                return False
            # sparse groups, registers per LDS hash-table slot: the smallest table (64 slots) must
            # hold every sketch's 2^p registers next to the slots (p = 11: one HLL per query)
            return 64 * ((1 + n) * 8 + nh * (1 << prog.hll_p)) <= 160 * 1024 - 256
        return prog.G * nh * (1 << prog.hll_p) <= PART_HLL_MAX_BYTES
    return True


# accumulator copies per wave for tiny dense key spaces (lanes l, l+C, l+2C.. share copy l % C; up
# to 64 = lane-private, no same-address LDS atomics) -- the LDS budget may halve it
MAX_NCOPY = 16
# whole-chunk fast path: a chunk entirely inside the scan's row range with no chunk-level bitmap
# prefilter walks its 64 words in order (every word's row mask all ones, then refined by the
# per-row filter) instead of the find-first-set / readlane chain over its non-empty words
FULL_CHUNKS = True
# a prefiltered chunk with at least this many non-empty words (of 64) also walks them in order,
# reading each word's mask by lane index (independent readlanes) and skipping all-empty steps;
# sparser chunks take the find-first-set chain over their non-empty words only (0: always chain)
DENSE_WORDS = 48
DENSE_WORDS_PACKED = 16  # (the same switch for kernels reading lane-interleaved packed columns)
# Count-only scans of tiny dense key spaces (TPC-H "Ship Date Range": count(*) by l_returnflag,
# l_linestatus over 150M rows) count in registers: per slot one 64-bit word of eight 8-bit fields,
# ``pc += (uint64)mine << (key * 8)`` per row (no LDS atomic -- every lane of a wave would otherwise
# hit the same few LDS words, serialized in the LDS atomic unit), unpacked into per-group u32
# counters at the end of each chunk (a lane sees <= 64 rows of a chunk, so no field overflows) and
# wave-reduced once into the accumulator table at the end.
COUNT_REGS = True
COUNT_REGS_MAX_G = 8


def count_regs(prog, mode: int) -> bool:
    return (COUNT_REGS and mode == D.M_DENSE_LDS and 0 < prog.G <= COUNT_REGS_MAX_G and not prog.nhll
            and bool(prog.aops) and all(a["kind"] == D.A_COUNT for a in prog.aops)
            and not getattr(prog, "presence_only", False))




# Dense LDS tables are sized for a power-of-two class of the group count, not the exact count: a
# dashboard's parameterizations differ mostly in how many values a key takes (a date range spans
# 3, 4 or 5 years -> 12, 16 or 20 groups), and with the count out of the code they share one
# kernel instead of compiling one per binding (~300 ms each, the BI plan's cold-start tail).  The
# exact count stays in the descriptor (d->G bounds the flush), and the class is used only when it
# keeps the same number of per-wave copies within the same LDS budget.
G_CLASS = True


def layout(prog, mode: int, U: int, hll_lds: bool, m: int, budget: int = 150 * 1024,
           regstage: bool = False, shared: bool = False) -> JitLayout:
    exact = _layout(prog, mode, U, hll_lds, m, budget, regstage, shared, int(prog.G))
    G = int(prog.G)
    if not G_CLASS or mode != D.M_DENSE_LDS or G <= 0 or count_regs(prog, mode):
        return exact
    gc = 1 << (G - 1).bit_length()
    if gc == G:
        return exact
    lay = _layout(prog, mode, U, hll_lds, m, budget, regstage, shared, gc)
    if lay.ncopy != exact.ncopy or (lay.total > budget and exact.total <= budget) or lay.total > 160 * 1024:
        return exact
    return lay


def _layout(prog, mode: int, U: int, hll_lds: bool, m: int, budget: int, regstage: bool, shared: bool,
            G: int) -> JitLayout:
    cols = col_infos(prog)
    nplanes = 0 if regstage else sum(2 if c.lg == 3 else 1 for c in cols.values() if not c.pw)
    need_bmw = _needs_word_bitmaps(prog)
    wave_bytes = U * nplanes * 256 + (len(prog.bm_leaves) * 512 if need_bmw else 0)
    wave_bytes = (wave_bytes + 15) // 16 * 16
    hll_bytes = prog.nhll * G * m if hll_lds else 0  # byte registers (hll_update8)
    stage = W * wave_bytes
    ncopy = 1
    acc_bytes = 0
    if mode == D.M_DENSE_LDS and shared:
        # key spaces too large for per-wave copies (thousands of groups, e.g. SSB brand x year):
        # ONE table per workgroup; lanes hitting the same group serialize in the LDS atomic unit,
        # which is still far cheaper than contending HBM atomics on a few hundred hot addresses
        acc_bytes = G * prog.nslots * 8
    elif mode == D.M_PART:
        acc_bytes = PART_HIST_BYTES  # the level-1 bucket histogram (sdo_device.h part_hist_add)
    elif mode == D.M_DENSE_LDS:
        base = G * prog.nslots * 8 * W
        ncopy = MAX_NCOPY
        while ncopy > 1 and base * ncopy + hll_bytes + stage > budget:
            ncopy //= 2
        acc_bytes = base * ncopy
    acc_off = 0
    hll_off = (acc_bytes + 15) // 16 * 16
    cache_off = (hll_off + hll_bytes + 15) // 16 * 16
    total = cache_off + stage
    return JitLayout(acc_off, acc_bytes, hll_off, hll_bytes, cache_off, wave_bytes, total, ncopy, regstage,
                     shared and mode == D.M_DENSE_LDS, G)


PRE_LDS_SELECTIVITY = 0.25


def prefer_regstage(prog) -> bool:
    """Staging choice measured on MI355X (tools/query_probe.py, SF100): VGPR staging wins for wide
    unfiltered payloads (TPC-H Q1: 1.9 vs 2.2 ms), LDS-DMA staging for word-filtered scans and tiny
    payloads (Q8: 0.14 vs 0.29 ms, 2-byte payload count: 0.46 vs 0.65 ms)."""
    if prog.filter_len and not prog.final_pre:
        return False
    # a selective chunk pre-filter (bitmap leaves) leaves a few rows per word: LDS-DMA staging
    # (TPC-H Q11's partitioned producer, 4% of rows: 3.46 -> 2.22 ms; tools/sql_probe.py A/B)
    n = max(1, int(getattr(getattr(prog, "ds", None), "num_rows", 0) or 1))
    if prog.pre_len and float(getattr(prog, "est_rows", n)) < PRE_LDS_SELECTIVITY * n:
        return False
    cols = col_infos(prog)
    return sum((c.pw / 8) if c.pw else (1 << c.lg) for i, c in cols.items() if i >= D.PAYLOAD_BASE) > 4


def _needs_word_bitmaps(prog) -> bool:
    spans = [(0, prog.filter_len)] if not prog.final_pre else []
    for a in prog.aops:
        if a.get("filt_len"):
            spans.append((a["filt_off"], a["filt_off"] + a["filt_len"]))
    return any(prog.fops[i][0] == D.F_BITMAP for a, b in spans for i in range(a, b))


def _lit(v: int) -> str:
    v = int(v)
    if v == -(2 ** 63):
        return "(-9223372036854775807LL - 1)"
    return f"{v}LL"


def _dlit(v: float) -> str:
    if v == float("inf"):
        return "__builtin_inf()"
    if v == float("-inf"):
        return "(-__builtin_inf())"
    return repr(float(v))


class _Gen:
    def __init__(self, prog, mode: int, U: int, hll_lds: bool, narrow4: bool, lay: JitLayout, m: int,
                 literals: bool = False):
        self.p = prog
        self.literals = literals
        self.nconst = 0
        self.regstage = lay.regstage
        self.mode = mode
        self.U = U
        self.hll_lds = hll_lds
        self.n4 = "true" if narrow4 else "false"
        self.lay = lay
        self.m = m
        self.cols = col_infos(prog)
        self.NP = sum(2 if c.lg == 3 else 1 for c in self.cols.values() if not c.pw)
        self.pre_lines: List[str] = []  # kernel-entry pointer / constant loads
        self._const_set = set()

    # ---------------------------------------------------------------- values
    def ival(self, idx: int) -> str:
        c = self.cols[idx]
        if c.pw:
            return f"(pk_field<{c.pw}>(xp{idx}[u], pks{idx}[u]) + {_lit(c.pbase)})"
        if self.regstage:
            return f"cv_int<{c.lg}, {'true' if c.sgn else 'false'}, {'true' if c.flt else 'false'}>(x{idx}[u])"
        return (f"ld_int<{c.lg}, {'true' if c.sgn else 'false'}, {'true' if c.flt else 'false'}, {self.n4}>"
                f"(wb + (u * {self.NP} + {c.plane}) * 256, lane)")

    def dval(self, idx: int) -> str:
        c = self.cols[idx]
        if c.pw:
            return f"((double){self.ival(idx)})"
        if self.regstage:
            return f"cv_dbl<{c.lg}, {'true' if c.sgn else 'false'}, {'true' if c.flt else 'false'}>(x{idx}[u])"
        return (f"ld_dbl<{c.lg}, {'true' if c.sgn else 'false'}, {'true' if c.flt else 'false'}, {self.n4}>"
                f"(wb + (u * {self.NP} + {c.plane}) * 256, lane)")

    # ---------------------------------------------------------------- query constants
    # Filter bounds, zone bounds, key bases / cards / strides and expression constants are read
    # from the descriptor (scalar loads once per kernel), not baked into the source: every
    # parameterization of one query shape -- another date range, nation, segment -- reuses ONE
    # compiled code object (a dashboard's distinct statements would otherwise each pay a hipRTC
    # compile), and the source hash keys only the shape.
    def const(self, name: str, expr: str, ctype: str = "int64_t", lit: Optional[str] = None) -> str:
        if lit is not None and (self.literals or JIT_LITERALS):
            return lit  # (A/B switch: the value baked into the source, one code object per value)
        if name[:2] in ("fl", "fh", "ff", "fg", "ec"):
            self.nconst += 1
        line = f"const {ctype} {name} = {expr};"
        if line not in self._const_set:
            self._const_set.add(line)
            self.pre_lines.append(line)
        return name

    # ---------------------------------------------------------------- filters
    def word_expr(self, lo: int, hi: int) -> str:
        st: List[str] = []
        for i in range(lo, hi):
            op, col, flags, a, b, fa, fb, bits = self.p.fops[i]
            if op == D.F_TRUE:
                st.append("(~0ull)")
            elif op == D.F_FALSE:
                st.append("(0ull)")
            elif op == D.F_BITMAP:
                st.append(f"uniform64(bmw[{int(a)} * 64 + wl[u]])")
            elif op in (D.F_ID_RANGE, D.F_INT_RANGE):
                # Bounds come from the descriptor (parameterizations share code), but an open side
                # (a one-sided range) is part of the shape and compiles away, and columns of <= 4
                # signed / <= 2 bytes compare in 32 bits against bounds clamped to int32 (the
                # clamped bound selects exactly the same rows of such a column).
                c = self.cols[col]
                narrow = not c.pw and not c.flt and (c.lg <= 1 or (c.lg == 2 and c.sgn))
                lo, hi = int(a), int(b)
                if op == D.F_ID_RANGE:
                    lo_open, hi_open = lo <= 0, False
                    hi_src = f"d->fops[{i}].hi - 1"  # exclusive -> inclusive
                else:
                    lo_open = lo == int(D.INT64_MIN) or (narrow and lo <= -(1 << 31))
                    hi_open = hi == int(D.INT64_MAX) or (narrow and hi >= (1 << 31) - 1)
                    hi_src = f"d->fops[{i}].hi"
                hi_incl = hi - 1 if op == D.F_ID_RANGE else hi
                if narrow:
                    c32 = lambda x: str(max(-(1 << 31), min((1 << 31) - 1, x)))  # noqa: E731
                    fl = self.const(f"fl{i}", f"clamp_i32(d->fops[{i}].lo)", "int32_t", c32(lo))
                    fh = self.const(f"fh{i}", f"clamp_i32({hi_src})", "int32_t", c32(hi_incl))
                    vdecl = f"const int32_t v = (int32_t)({self.ival(col)});"
                else:
                    fl = self.const(f"fl{i}", f"d->fops[{i}].lo", lit=_lit(lo))
                    fh = self.const(f"fh{i}", hi_src, lit=_lit(hi_incl))
                    vdecl = f"const int64_t v = {self.ival(col)};"
                conds = ([] if lo_open else [f"v >= {fl}"]) + ([] if hi_open else [f"v <= {fh}"])
                if not conds:
                    st.append("(~0ull)")
                else:
                    st.append(f"({{ {vdecl} (uint64_t)__ballot({' && '.join(conds)}); }})")
            elif op == D.F_IN_SET:
                self.pre_lines.append(f"const uint64_t* inset{i} = (const uint64_t*)" +
                                      f"d->fops[{i}].bits;")
                st.append(f"({{ const int64_t v = {self.ival(col)}; "
                          f"(uint64_t)__ballot((inset{i}[((uint64_t)v) >> 6] >> (v & 63)) & 1ull); }})")
            elif op == D.F_FLT_RANGE:
                lo_c = ">" if flags & 1 else ">="
                hi_c = "<" if flags & 2 else "<="
                fl = self.const(f"ff{i}", f"d->fops[{i}].flo", "double", _dlit(fa))
                fh = self.const(f"fg{i}", f"d->fops[{i}].fhi", "double", _dlit(fb))
                st.append(f"({{ const double v = {self.dval(col)}; "
                          f"(uint64_t)__ballot(v {lo_c} {fl} && v {hi_c} {fh}); }})")
            elif op == D.F_EXPR:
                lo_c = ">" if flags & 1 else ">="
                hi_c = "<" if flags & 2 else "<="
                ev = self.expr(self.p.eops[int(a):int(a) + int(b)], int(a))
                fl = self.const(f"ff{i}", f"d->fops[{i}].flo", "double", _dlit(fa))
                fh = self.const(f"fg{i}", f"d->fops[{i}].fhi", "double", _dlit(fb))
                st.append(f"({{ const double v = {ev}; "
                          f"(uint64_t)__ballot(v {lo_c} {fl} && v {hi_c} {fh}); }})")
            elif op in (D.F_AND, D.F_OR):
                y, x = st.pop(), st.pop()
                st.append(f"({x} {'&' if op == D.F_AND else '|'} {y})")
            elif op == D.F_NOT:
                st.append(f"(~{st.pop()})")
            else:
                raise ValueError(f"opcode {op} not supported in jit word filter")
        return st[-1] if st else "(~0ull)"

    def chunk_expr(self) -> str:
        st: List[str] = []
        p = self.p
        for i in range(p.pre_off, p.pre_off + p.pre_len):
            op, col, flags, a, b, fa, fb, bits = p.fops[i]
            if op == D.F_BITMAP:
                st.append(f"lw{int(a)}")
            elif op == D.F_TRUE:
                st.append("(~0ull)")
            elif op == D.F_FALSE:
                st.append("(0ull)")
            elif op in (D.F_AND, D.F_OR):
                y, x = st.pop(), st.pop()
                st.append(f"({x} {'&' if op == D.F_AND else '|'} {y})")
            elif op == D.F_NOT:
                st.append(f"(~{st.pop()})")
            else:
                raise ValueError(f"opcode {op} in chunk-level program")
        return st[-1] if st else "(~0ull)"

    # ---------------------------------------------------------------- expression VM -> C++
    def expr(self, eops, off: int = 0) -> str:
        st: List[str] = []
        for j, (op, col, c) in enumerate(eops):
            if op == D.E_LUT:
                # dictionary-domain value table: pointer read from the descriptor, so the JIT
                # source (and its cache key) does not depend on the allocation
                st.append(f"(((const double*)__double_as_longlong(d->eops[{off + j}].c))"
                          f"[{self.ival(col)}])")
            elif op == D.E_COL:
                v = self.dval(col)
                st.append(f"({v} * {self.const(f'ec{off + j}', f'd->eops[{off + j}].c', 'double', _dlit(c))})"
                          if c != 0.0 else f"({v})")
            elif op == D.E_CONST:
                st.append(f"({self.const(f'ec{off + j}', f'd->eops[{off + j}].c', 'double', _dlit(c))})")
            elif op == D.E_NEG:
                st.append(f"(-{st.pop()})")
            elif op == D.E_ABS:
                st.append(f"fabs({st.pop()})")
            elif op in (D.E_FLOOR, D.E_CEIL, D.E_SQRT, D.E_LOG, D.E_EXP):
                fn = {D.E_FLOOR: "floor", D.E_CEIL: "ceil", D.E_SQRT: "sqrt", D.E_LOG: "log", D.E_EXP: "exp"}[op]
                st.append(f"{fn}({st.pop()})")
            elif op in (D.E_MOD, D.E_PMOD, D.E_POW):
                y, x = st.pop(), st.pop()
                if op == D.E_MOD:
                    st.append(f"fmod({x}, {y})")
                elif op == D.E_POW:
                    st.append(f"pow({x}, {y})")
                else:
                    st.append(f"([](double a_, double b_) {{ const double m_ = fmod(a_, b_); "
                              f"return m_ < 0.0 ? fmod(m_ + b_, b_) : m_; }})({x}, {y})")
            else:
                y, x = st.pop(), st.pop()
                sym = {D.E_ADD: "+", D.E_SUB: "-", D.E_MUL: "*", D.E_DIV: "/"}.get(op)
                if sym:
                    st.append(f"({x} {sym} {y})")
                else:
                    st.append(f"{'fmin' if op == D.E_MIN else 'fmax'}({x}, {y})")
        return st[-1]

    def stage_words(self, o: List[str], cols, wl: str, dst: str, ind: str = "      ",
                    j0: Optional[int] = None) -> None:
        """Load the given columns of U whole 64-row words through the per-chunk buffer resources
        (``rs<i>``) -- into VGPR arrays ``x<i>[u]`` (register staging) or LDS planes (DMA);
        ``wl`` names the per-u word-in-chunk array.  Bit-packed columns (segment/packed.py
        lane-interleaved streams) land as a 64-bit window ``xp<i>[u]`` + field shift ``pks<i>[u]``:
        for words ``g_ * 32 + j0 + u`` (``j0`` static) as the ``U W / 32`` (+1) coalesced stream
        dwords of the run with compile-time field offsets, else two dword loads per word."""
        U, NP = self.U, self.NP
        pk = [i for i in cols if self.cols[i].pw]
        cols = [i for i in cols if not self.cols[i].pw]
        for i in pk:  # bit-packed columns: straight into registers in either staging mode
            W = self.cols[i].pw
            o.append(f"{ind}uint64_t xp{i}[{U}]; uint32_t pks{i}[{U}];")
            if j0 is None:
                o.append(f"#pragma unroll\n{ind}for (int u = 0; u < {U}; ++u) {{")
                o.append(f"{ind}  const uint32_t b_ = ((uint32_t){wl}[u] & 31u) * {W}u;")
                soff = f"((uint32_t){wl}[u] >> 5) * {256 * W}u + ((b_ >> 5) << 8)"
                if 32 % W == 0:  # (a field never straddles a stream dword: one load)
                    o.append(f"{ind}  xp{i}[u] = __builtin_amdgcn_raw_buffer_load_b32(rs{i}, lq4, {soff}, 0);")
                else:
                    o.append(f"{ind}  xp{i}[u] = ld_il(rs{i}, {soff}, lq4);")
                o.append(f"{ind}  pks{i}[u] = b_ & 31u;")
                o.append(f"{ind}}}")
                continue
            k0, k1 = (j0 * W) >> 5, ((j0 + U) * W - 1) >> 5
            n = k1 - k0 + 1
            o.append(f"{ind}uint32_t xd{i}[{n + 1}];")
            o.append(f"#pragma unroll\n{ind}for (int k = 0; k < {n}; ++k) xd{i}[k] = __builtin_amdgcn_raw_buffer_load_b32("
                     f"rs{i}, lq4, (uint32_t)g_ * {256 * W}u + ({k0} + k) * 256u, 0);")
            o.append(f"{ind}xd{i}[{n}] = 0u;")
            o.append(f"#pragma unroll\n{ind}for (int u = 0; u < {U}; ++u) {{")
            o.append(f"{ind}  const int b_ = ({j0} + u) * {W} - {32 * k0};")
            o.append(f"{ind}  xp{i}[u] = (uint64_t)xd{i}[b_ >> 5] | ((uint64_t)xd{i}[(b_ >> 5) + 1] << 32);")
            o.append(f"{ind}  pks{i}[u] = (uint32_t)(b_ & 31);")
            o.append(f"{ind}}}")
        if not cols:
            return
        if self.regstage:
            for i in cols:
                o.append(f"{ind}{'uint64_t' if self.cols[i].lg == 3 else 'uint32_t'} x{i}[{U}];")
            o.append(f"#pragma unroll\n{ind}for (int u = 0; u < {U}; ++u) {{")
            for i in cols:
                c = self.cols[i]
                o.append(f"{ind}  x{i}[u] = ld_b<{c.lg}>(rs{i}, (uint32_t){wl}[u] << {6 + c.lg}, lo{c.lg});")
            o.append(f"{ind}}}")
            return
        o.append(f"#pragma unroll\n{ind}for (int u = 0; u < {U}; ++u) {{")
        for i in cols:
            c = self.cols[i]
            o.append(f"{ind}  dma_b<{c.lg}>(rs{i}, (uint32_t){wl}[u] << {6 + c.lg}, lo{c.lg}, "
                     f"{dst} + (u * {NP} + {c.plane}) * 256);")
        o.append(f"{ind}}}")

    # ---------------------------------------------------------------- whole kernel
    def _part_record(self, body: List[str]) -> None:
        """M_PART producer: the row becomes a partition record (ops/csrc/partition.hip) instead of a
        table update -- u32 key, then every aggregator's value (``part_fields``: implicit / i32 /
        i64 words; a row an aggregator's own filter rejects carries the slot's identity).  Records
        are appended to the chunk's own region (chunk c owns records [4096 c, 4096 c + 4096)), at
        the wave's running offset plus the lane's rank among the active lanes: consecutive lanes
        write consecutive records, no atomics; the split kernels then bucket them."""
        p = self.p
        body.append("        const bool mine = act[u];")
        body.append("        const uint64_t am_ = __ballot(mine);")
        fields = part_fields(p, self.cols)
        hdr = part_record_words(p)
        rw = hdr + sum(w for _, w in fields) + part_hll_count(p)
        if hdr == 3:
            # 64-bit key: partitioned by the top bits of a multiplicative hash
            body.append("        const uint32_t pk_ = (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> 32);")
        else:
            body.append("        const uint32_t pk_ = (uint32_t)key;")
        body.append("        if (mine) {")
        body.append(f"          uint32_t* o_ = precs + (uint64_t)(cbase + woff + (uint32_t)__popcll(am_ & lmlt)) * {rw}u;")
        body.append("          o_[0] = pk_;")
        if hdr == 3:
            body.append("          o_[1] = (uint32_t)key; o_[2] = (uint32_t)((uint64_t)key >> 32);")
        w = hdr
        fi = 0
        for ai, a in enumerate(p.aops):
            if a["kind"] in (D.A_HLL, D.A_HLL_CODE, D.A_HLL_STORED):
                continue
            slot, width = fields[fi]
            fi += 1
            if width == 0:
                continue
            cond = None
            if a.get("filt_len"):
                cond = f"((({self.word_expr(a['filt_off'], a['filt_off'] + a['filt_len'])}) >> lane) & 1ull)"
            val = f"v{ai}_[u]"
            if a["kind"] == D.A_COUNT:
                val = f"({cond} ? 1LL : 0LL)" if cond else "1LL"
            elif cond:
                val = f"({cond} ? {val} : (int64_t){_lit(p.slots[slot][1])})"
            if width == 1:
                body.append(f"          o_[{w}] = (uint32_t)(int32_t)({val});")
            else:
                body.append(f"          {{ const uint64_t x_ = (uint64_t)({val}); o_[{w}] = (uint32_t)x_; "
                            f"o_[{w + 1}] = (uint32_t)(x_ >> 32); }}")
            w += width
        for ai, a in enumerate(p.aops):
            # HLL: the row's (bucket << 8 | rho) word (rho 0: no update -- a row its filter rejects)
            if a["kind"] not in D.HLL_KINDS:
                continue
            val = f"v{ai}_[u]"
            if a["kind"] == D.A_HLL_CODE:  # precomputed code plane: bucket << 5 | rho
                code = f"(((((uint32_t){val}) >> 5) << 8) | ((uint32_t){val} & 31u))"
            else:
                code = f"({{ uint32_t b_, r_; hll_bucket_rho({val}, {_lit(a.get('salt', 0))}, {p.hll_p}, b_, r_); " \
                       f"(b_ << 8) | r_; }})"
            if a.get("filt_len"):
                fx = self.word_expr(a["filt_off"], a["filt_off"] + a["filt_len"])
                code = f"(((({fx}) >> lane) & 1ull) ? {code} : 0u)"
            body.append(f"          o_[{w}] = {code};")
            w += 1
        for ai, a in enumerate(p.aops):
            # stored sketch: the row id (its CSR run of stored pairs), all-ones when filtered out
            if a["kind"] != D.A_HLL_STORED:
                continue
            rid = f"(uint32_t)(v{ai}_[u])"
            if a.get("filt_len"):
                fx = self.word_expr(a["filt_off"], a["filt_off"] + a["filt_len"])
                rid = f"(((({fx}) >> lane) & 1ull) ? {rid} : 0xffffffffu)"
            body.append(f"          o_[{w}] = {rid};")
            w += 1
        body.append("        }")
        # (dense keys come in runs: the clustered add; hashes are uniform)
        body.append(f"        if (phout) part_hist_add(phist, (pk_ >> pshift) & pmask, mine, {'false' if hdr == 3 else 'true'});")
        body.append("        woff += (uint32_t)__popcll(am_);")

    def _words_tail(self, fcols, word_filter, mode: int, U: int, stage: List[str], body: List[str],
                    j0: Optional[int] = None) -> List[str]:
        """The per-step tail of a word loop (wl / m set): the per-row word filter, the empty-step
        skip, then the staged loads and updates."""
        out: List[str] = []
        if word_filter is not None:
            if fcols:
                dma = not self.regstage and any(not self.cols[i].pw for i in fcols)
                if dma:
                    out.append('      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");')
                self.stage_words(out, fcols, "wl", "wb", j0=j0)
                if dma:
                    out.append('      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
            out.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) m[u] &= {word_filter};")
        out.append("      uint64_t any = 0;")
        out.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) any |= m[u];")
        out.append("      if (any == 0) continue;")
        if mode == D.M_MASK:
            out.append("      if (lane == 0) {")
            out.append("        unsigned long long cnt = 0;")
            out.append(f"#pragma unroll\n        for (int u = 0; u < {U}; ++u) {{")
            out.append("          if (m[u]) ((uint64_t*)d->out_mask)[cw0 + wl[u]] = m[u];")
            out.append("          cnt += __popcll(m[u]);")
            out.append("        }")
            out.append("        atomicAdd((unsigned long long*)d->out_count, cnt);")
            out.append("      }")
        else:
            out.extend(stage + body)
        return out

    def source(self, name: str) -> str:
        p, U, NP, lay = self.p, self.U, self.NP, self.lay
        mode = self.mode
        L: List[str] = []
        fcols = [i for i in sorted(self.cols) if i < D.PAYLOAD_BASE]
        pcols = [i for i in sorted(self.cols) if i >= D.PAYLOAD_BASE]
        need_bmw = _needs_word_bitmaps(p)
        word_filter = None if p.final_pre else self.word_expr(0, p.filter_len)
        pre = self.chunk_expr() if p.pre_len else None
        G, NS = p.G, p.nslots
        GL = lay.G or G  # (the LDS table's size class; exact G only for the unrolled count registers)
        NCT = 1 if lay.shared else W * lay.ncopy
        creg = count_regs(p, mode)
        cslots = sorted({a["slot"] for a in p.aops}) if creg else []
        for i in sorted(self.cols):
            L.append(f"  const unsigned char* c{i} = (const unsigned char*)d->cols[{i}].ptr;")
        for j, (row, stride, count) in enumerate(p.bm_leaves):
            # (VGPR-resident: read once per chunk with a per-lane address anyway)
            L.append(f"  const uint64_t* bm{j} = (const uint64_t*)" +
                     f"d->bm_bits[{j}];")
        for k, kc in enumerate(p.keys):
            if kc.kind == D.K_REMAP or (kc.kind == D.K_TIME and getattr(kc, "tlut", None) is not None):
                L.append(f"  const int32_t* rm{k} = (const int32_t*)d->kops[{k}].remap;")
        for z in range(len(p.zones)):
            L.append(f"  const int32_t* zmin{z} = (const int32_t*)d->zones[{z}].zmin;")
            L.append(f"  const int32_t* zmax{z} = (const int32_t*)d->zones[{z}].zmax;")
            L.append(f"  const int64_t zlo{z} = d->zones[{z}].lo;")
            L.append(f"  const int64_t zhi{z} = d->zones[{z}].hi;")
        for ai, a in enumerate(p.aops):
            if a["kind"] in D.HLL_KINDS:
                if self.hll_lds and mode == D.M_DENSE_LDS:
                    L.append(f"  unsigned char* hll{ai} = lds + {lay.hll_off + a['hll'] * GL * self.m};")
                else:
                    L.append(f"  unsigned char* hll{ai} = (unsigned char*)d->aops[{ai}].hll_regs;")
            elif a["kind"] == D.A_HLL_STORED:
                L.append(f"  unsigned char* hll{ai} = (unsigned char*)d->aops[{ai}].hll_regs;")
                L.append(f"  const int64_t* sko{ai} = (const int64_t*)d->aops[{ai}].sk_off;")
                L.append(f"  const int32_t* skv{ai} = (const int32_t*)d->aops[{ai}].sk_val;")
        def mk_stage(j0: Optional[int]) -> List[str]:
            st = ["      // ---- payload staging (whole words) ----", f"      bool act[{U}];",
                  f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) act[u] = (m[u] >> lane) & 1ull;"]
            if pcols:
                dma = not self.regstage and any(not self.cols[i].pw for i in pcols)
                if dma:
                    st.append('      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");')
                self.stage_words(st, pcols, "wl", "wb", j0=j0)
                if dma:
                    st.append('      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
            return st

        # ---------------- per-word processing
        stage = mk_stage(None)
        def _mk_body(U: int) -> List[str]:
            body = []
            # phase 1: every staged read for the U words (keys + aggregator inputs) -- straight-line
            # LDS reads the compiler can issue back to back; phase 2 applies the updates.
            body.append(f"      uint64_t key_[{U}];")
            vals: Dict[int, str] = {}
            for ai, a in enumerate(p.aops):
                body.append(f"      int64_t v{ai}_[{U}];")
            body.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) {{")
            body.append("        uint64_t key = 0;")
            for k, kc in enumerate(p.keys):
                v = self.ival(kc.col_idx)
                # stride / base / card from the descriptor (query constants); for LDS tables the
                # layout (G) is part of the shape anyway
                ks = self.const(f"ks{k}", f"(uint64_t)d->kops[{k}].stride", "uint64_t", f"{int(kc.stride)}ull")
                kb = self.const(f"kb{k}", f"d->kops[{k}].base", lit=_lit(kc.base))
                kn = self.const(f"kn{k}", f"d->kops[{k}].card", lit=_lit(kc.card))
                if kc.kind == D.K_ID and kc.base:  # shard-local key window (engine/executor.py ShardWindow)
                    body.append(f"        key += (uint64_t)((int64_t)({v}) - {kb}) * {ks};")
                elif kc.kind == D.K_ID:
                    body.append(f"        key += (uint64_t)({v}) * {ks};")
                elif kc.kind == D.K_REMAP:
                    body.append(f"        key += (uint64_t)rm{k}[{v}] * {ks};")
                elif kc.kind == D.K_TIME and getattr(kc, "tlut", None) is not None:
                    n = len(kc.tlut)  # precomputed key per raw time value (engine/lower.py _attach_time_lut)
                    body.append(f"        {{ int64_t i_ = (int64_t)({v}) - {_lit(kc.tlut_lo)};")
                    body.append(f"          i_ = i_ < 0 ? 0 : (i_ >= {n} ? {n - 1} : i_);")
                    body.append(f"          key += (uint64_t)rm{k}[i_] * {ks}; }}")
                elif kc.kind == D.K_TIME:
                    ktz = self.const(f"ktz{k}", f"d->kops[{k}].tz_ms", lit=_lit(kc.tz_ms))
                    kpm = self.const(f"kpm{k}", f"d->kops[{k}].period_ms", lit=_lit(kc.period_ms or 1))
                    kor = self.const(f"kor{k}", f"d->kops[{k}].origin_ms", lit=_lit(kc.origin_ms))
                    body.append(f"        {{ int64_t t = time_field_t<{kc.tfield}>(({v}) * {_lit(p.ds.time_unit_ms)} + "
                                f"{ktz}, {kpm}, {kor}) - {kb};")
                    body.append(f"          t = t < 0 ? 0 : (t >= {kn} ? {kn} - 1 : t);")
                    body.append(f"          key += (uint64_t)t * {ks}; }}")
                else:
                    body.append(f"        {{ int64_t t = ({v}) - {kb};")
                    body.append(f"          t = t < 0 ? 0 : (t >= {kn} ? {kn} - 1 : t);")
                    body.append(f"          key += (uint64_t)t * {ks}; }}")
            body.append("        key_[u] = key;")
            for ai, a in enumerate(p.aops):
                kind = a["kind"]
                if kind in D.HLL_KINDS:
                    val = self.ival(a["col"])
                elif kind in (D.A_HLL_STORED, D.A_ROWID):
                    val = "((cw0 + wl[u]) * 64 + lane)"  # the row (a stored sketch's CSR run / emitted id)
                elif kind == D.A_THETA:
                    # the thetaSketch hash of the row's value: theta_hash (segment/ingest.py) in-kernel
                    val = (f"(int64_t)(mix64((uint64_t)(int64_t)({self.ival(a['col'])}) ^ 0x5BD1E995ull) & "
                           "0x3FFFFFFFFFFFFFFFull)")
                elif kind == D.A_COUNT:
                    val = "1LL"
                elif kind == D.A_SUM_X:
                    val = f"(int64_t)rint({self.expr(a['expr'], a.get('expr_off', 0))})"
                elif kind in (D.A_SUM_F, D.A_MIN_F, D.A_MAX_F):
                    dv = self.expr(a["expr"], a.get("expr_off", 0)) if a.get("expr") else self.dval(a["col"])
                    val = f"__double_as_longlong({dv})" if kind == D.A_SUM_F else f"f2ord({dv})"
                else:
                    val = self.ival(a["col"])
                body.append(f"        v{ai}_[u] = {val};")
            body.append("      }")
            body.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) {{")
            body.append("        const uint64_t key = key_[u];")
            if mode == D.M_PART:
                self._part_record(body)
            elif mode == D.M_HASH:
                body.append("        int64_t slot = act[u] ? hash_slot(hkeys, hcap, key, overflow) : -1;")
                body.append("        const bool mine = act[u] && slot >= 0;")
            else:
                body.append("        const int64_t slot = (int64_t)key;")
                body.append("        const bool mine = act[u];")
                if mode == D.M_DENSE_GLOBAL and getattr(p, "touch_table", False):
                    # first-touch byte table (engine/device_exec.py): every group a qualifying row
                    # reaches is marked with a plain byte store (same-value races are benign); the
                    # touched groups compact from this table instead of the accumulator table, and only
                    # they are re-initialised after the run (no full-table fill per execution)
                    body.append("        if (mine) ((unsigned char*)d->out_mask)[slot] = (unsigned char)1;")
            for ai, a in enumerate(p.aops if mode != D.M_PART else []):
                cond = "mine"
                if a.get("filt_len"):
                    fx = self.word_expr(a["filt_off"], a["filt_off"] + a["filt_len"])
                    body.append(f"        const bool f{ai} = mine && ((({fx}) >> lane) & 1ull);")
                    cond = f"f{ai}"
                kind = a["kind"]
                val = f"v{ai}_[u]"
                wide = getattr(p, "hll32", False) and not (self.hll_lds and mode == D.M_DENSE_LDS)
                if kind == D.A_HLL_CODE:
                    # precomputed (bucket, rho) plane (segment/hllcode.py): no per-row hash
                    ix = f"((uint64_t)slot << {p.hll_p}) + ((uint32_t){val} >> 5)"
                    fn = "hll_max32((uint32_t*)" if wide else "hll_max8("
                    body.append(f"        if ({cond}) {fn}hll{ai}, {ix}, (uint32_t){val} & 31u);")
                    continue
                if kind == D.A_HLL:
                    if wide:  # global u32 registers (engine/device_exec.py narrows them after the scan)
                        body.append(f"        if ({cond}) hll_update32((uint32_t*)hll{ai}, slot, {p.hll_p}, {val}, "
                                    f"{_lit(a.get('salt', 0))});")
                    else:
                        body.append(f"        if ({cond}) hll_update8(hll{ai}, slot, {p.hll_p}, {val}, "
                                    f"{_lit(a.get('salt', 0))});")
                    continue
                if kind == D.A_HLL_STORED:
                    fn = "hll_merge_csr32((uint32_t*)" if getattr(p, "hll32", False) else "hll_merge_csr("
                    body.append(f"        if ({cond}) {fn}hll{ai}, slot, {p.hll_p}, sko{ai}, skv{ai}, {val});")
                    continue
                s = a["slot"]
                op = p.slots[s][0]
                if creg:  # packed 8-bit register counters (COUNT_REGS)
                    body.append(f"        pc{s} += (uint64_t)({cond}) << ((uint32_t)key << 3);")
                    continue
                if mode == D.M_DENSE_LDS:
                    tgt = f"acc + (slot * {NS} + {s}) * {NCT} + copy"
                else:
                    tgt = f"gacc + slot * {NS} + {s}"
                if getattr(p, "presence_only", False) and mode == D.M_DENSE_GLOBAL and kind == D.A_COUNT and NS == 1:
                    # existence only (nested inner level, SELECT DISTINCT): a plain vector store of 1
                    # instead of an HBM read-modify-write atomic per row (same-value races are benign);
                    # with presence_bytes the table is one byte per group
                    if getattr(p, "presence_bytes", False):
                        body.append(f"        if ({cond}) ((unsigned char*)gacc)[slot] = (unsigned char)1;")
                    else:
                        body.append(f"        if ({cond}) *({tgt}) = 1ull;")
                    continue
                body.append(f"        if ({cond}) acc_update<{op}>({tgt}, {val});")
            body.append("      }")
            return body

        body = _mk_body(U)
        # ---------------- kernel text
        out = []
        out.append('#include "sdo_device.h"')
        out.append("using namespace sdo;")
        out.append("using namespace sdo::dev;")
        out.append(f'extern "C" __global__ __launch_bounds__({W * 64}) void {name}(const ScanDesc* __restrict__ d) {{')
        out.append("  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];")
        out.append("  const int lane = threadIdx.x & 63;")
        out.append("  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
        for lg in sorted({c.lg for c in self.cols.values() if not c.pw}):
            out.append(f"  const uint32_t lo{lg} = (uint32_t)lane << {lg};")
        if any(c.pw for c in self.cols.values()):
            out.append("  const uint32_t lq4 = (uint32_t)lane << 2;")
        out.append(f"  unsigned char* wb = lds + {lay.cache_off} + wave * {lay.wave_bytes};")
        stage_bytes = 0 if self.regstage else U * NP * 256
        out.append(f"  uint64_t* bmw = (uint64_t*)(wb + {stage_bytes});")
        out.append("  uint64_t* acc = (uint64_t*)lds;")
        if lay.shared:
            out.append("  const int copy = 0;")
        else:
            out.append(f"  const int copy = wave * {lay.ncopy} + (lane & {lay.ncopy - 1});")
        out.append("  uint64_t* gacc = (uint64_t*)d->out_acc;")
        out.append("  uint64_t* hkeys = (uint64_t*)d->out_keys;")
        out.append("  const int64_t hcap = d->hash_cap;")
        out.append("  int* overflow = (int*)d->overflow;")
        out.append("  (void)bmw; (void)acc; (void)copy; (void)gacc; (void)hkeys; (void)hcap; (void)overflow;")
        out.extend(L)
        out.extend("  " + x for x in self.pre_lines)
        if mode == D.M_PART:
            out.append("  uint32_t* precs = (uint32_t*)d->part_recs;")
            out.append("  uint32_t* pend = (uint32_t*)d->part_counts;  // end offset of each chunk's records")
            out.append("  const uint64_t lmlt = (1ull << lane) - 1ull;")
            # level-1 bucket histogram of this block's records (sdo_device.h part_hist_add), and
            # the block's chunk positions in workgroup order (part_positions)
            out.append("  uint32_t* phist = (uint32_t*)lds;")
            out.append("  uint32_t* phout = (uint32_t*)d->part_base;")
            out.append("  const int pshift = d->part_shift;")
            out.append("  const uint32_t pmask = ((uint32_t)d->part_n - 1u) & (PART_HIST_BUCKETS - 1u);")
            out.append(f"  for (int i = threadIdx.x; i < PART_HIST_BUCKETS; i += {W * 64}) phist[i] = 0u;")
            out.append("  __syncthreads();")
            out.append(f"  const int64_t tw_ = (int64_t)gridDim.x * {W};")
            out.append(f"  int64_t ppos = (int64_t)blockIdx.x * ((d->total_chunks + tw_ - 1) / tw_) * {W} + wave;"
                       f"  // += {W} per chunk")
        if mode == D.M_DENSE_LDS:
            out.append(f"  for (int i = threadIdx.x; i < {GL * NS * NCT}; i += {W * 64}) {{")
            inits = ", ".join(_lit(init) for _, init in p.slots)
            out.append(f"    constexpr int64_t init[{NS}] = {{{inits}}};")
            out.append(f"    acc[i] = (uint64_t)init[(i / {NCT}) % {NS}];")
            out.append("  }")
            if self.hll_lds and p.nhll:
                out.append(f"  for (int i = threadIdx.x; i < {lay.hll_bytes // 4}; i += {W * 64}) "
                           f"((uint32_t*)(lds + {lay.hll_off}))[i] = 0u;")
            out.append("  __syncthreads();")
        for s in cslots:
            out.append(f"  uint64_t pc{s} = 0;")
            out.append("  " + " ".join(f"uint32_t cn{s}_{g} = 0;" for g in range(G)))
        out.append(f"  const int64_t total_waves = (int64_t)gridDim.x * {W};")
        out.append(f"  const int64_t gw = (int64_t)blockIdx.x * {W} + wave;")
        out.append("  const int64_t num_rows = d->num_rows;")
        out.append("  const int nranges = d->nranges;")
        out.append("  for (int64_t c = gw; c < d->total_chunks; c += total_waves) {")
        if mode == D.M_PART:
            out.append(f"    const uint32_t cbase = (uint32_t)c * {D.CHUNK_ROWS}u;")
            out.append("    uint32_t woff = 0;")
            out.append("    const int64_t cpos = phout ? ppos : c;  // (emit / theta producers: chunk order)")
            out.append(f"    ppos += {W};")
            out.append("    if (lane == 0) pend[cpos] = cbase;  // (a skipped chunk holds no records)")
        out.append("    int r = 0;")
        out.append("    int64_t cc = c;")
        out.append("    while (r < nranges - 1 && cc >= d->ranges[r].nchunks) { cc -= d->ranges[r].nchunks; ++r; }")
        out.append("    const int64_t kchunk = d->ranges[r].chunk_begin + cc;")
        out.append(f"    int64_t clo = kchunk * {D.CHUNK_ROWS}, chi = clo + {D.CHUNK_ROWS};")
        out.append("    if (clo < d->ranges[r].lo) clo = d->ranges[r].lo;")
        out.append("    if (chi > d->ranges[r].hi) chi = d->ranges[r].hi;")
        out.append("    if (chi > num_rows) chi = num_rows;")
        out.append("    if (chi <= clo) continue;")
        for z, (dim, zlo, zhi) in enumerate(p.zones):
            out.append(f"    if ((int64_t)zmax{z}[kchunk] < zlo{z} || (int64_t)zmin{z}[kchunk] >= zhi{z}) continue;")
        out.append(f"    const int64_t cw0 = kchunk * {D.CHUNK_WORDS};")
        out.append(f"    const int64_t crow0 = kchunk * {D.CHUNK_ROWS};")
        out.append(f"    const int64_t crows = num_rows - crow0 < {D.CHUNK_ROWS} ? num_rows - crow0 : {D.CHUNK_ROWS};")
        staged = (fcols if word_filter is not None else []) + (pcols if mode != D.M_MASK else [])
        for i in staged:
            if self.cols[i].pw:
                out.append(f"    const __amdgpu_buffer_rsrc_t rs{i} = chunk_rsrc_pk(c{i}, kchunk, {self.cols[i].pw});")
            else:
                out.append(f"    const __amdgpu_buffer_rsrc_t rs{i} = chunk_rsrc(c{i}, crow0, crows, {self.cols[i].lg});")
        out.append("    const int64_t my_r0 = (cw0 + lane) * 64;")
        out.append("    const int64_t lo_off = clo - my_r0, hi_off = chi - my_r0;")
        out.append("    uint64_t pre = range_bits((int)(lo_off < 0 ? 0 : (lo_off > 64 ? 64 : lo_off)),")
        out.append("                              (int)(hi_off < 0 ? 0 : (hi_off > 64 ? 64 : hi_off)));")
        for j, (row, stride, count) in enumerate(p.bm_leaves):
            if count == 1:
                out.append(f"    const uint64_t lw{j} = bm{j}[cw0 + lane];")
            else:
                out.append(f"    uint64_t lw{j} = 0;")
                out.append(f"    for (int k = 0; k < {count}; ++k) lw{j} |= bm{j}[(int64_t)k * {stride} + cw0 + lane];")
            if need_bmw:
                out.append(f"    bmw[{j} * 64 + lane] = lw{j};")
        if pre:
            out.append(f"    pre &= {pre};")
        out.append("    uint64_t nz = __ballot(pre != 0ull);")
        full = FULL_CHUNKS and not pre and mode in (D.M_DENSE_LDS, D.M_DENSE_GLOBAL, D.M_HASH)
        # whole-chunk walks over a bit-packed column run as static runs of U words per 32-word
        # stream group: each run's stream dwords are U W / 32 (+1) coalesced loads with
        # compile-time field offsets (segment/packed.py); `continue` leaves only its own run
        static = U >= 4 and 32 % U == 0 and any(self.cols[i].pw for i in staged)

        def whole_chunk(mask: str) -> None:
            if static:
                out.append("    for (int g_ = 0; g_ < 2; ++g_) {")
                for j0 in range(0, 32, U):
                    out.append("    do {")
                    out.append(f"      int wl[{U}];")
                    out.append(f"      uint64_t m[{U}];")
                    out.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) {{ wl[u] = g_ * 32 + {j0} + u; "
                               f"m[u] = {mask}; }}")
                    out.extend(self._words_tail(fcols, word_filter, mode, U, mk_stage(j0), body, j0=j0))
                    out.append("    } while (0);")
                out.append("    }")
                return
            out.append(f"    for (int w0_ = 0; w0_ < {D.CHUNK_WORDS}; w0_ += {U}) {{")
            out.append(f"      int wl[{U}];")
            out.append(f"      uint64_t m[{U}];")
            out.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) {{ wl[u] = w0_ + u; m[u] = {mask}; }}")
            out.extend(self._words_tail(fcols, word_filter, mode, U, stage, body))
            out.append("    }")

        if full:
            out.append(f"    if (clo == crow0 && chi == crow0 + {D.CHUNK_ROWS}) {{")
            whole_chunk("~0ull")
            out.append("    } else {")
        dense = DENSE_WORDS > 0 and bool(pre) and mode in (D.M_DENSE_LDS, D.M_DENSE_GLOBAL, D.M_HASH)
        if dense:
            # a static whole-chunk walk costs ~2W stream loads per packed column; the sparse walk
            # two per column and nonzero word -- with packed columns it wins from far fewer words
            out.append(f"    if (__popcll(nz) >= {DENSE_WORDS_PACKED if static else DENSE_WORDS}) {{")
            whole_chunk("readlane64(pre, wl[u])")
            out.append("    } else {")
        out.append("    while (nz) {")
        out.append(f"      int wl[{U}];")
        out.append(f"      uint64_t m[{U}];")
        out.append(f"#pragma unroll\n      for (int u = 0; u < {U}; ++u) {{")
        out.append("        if (nz) { wl[u] = __builtin_ctzll(nz); nz &= nz - 1ull; m[u] = readlane64(pre, wl[u]); }")
        out.append("        else { wl[u] = 0; m[u] = 0ull; }")
        out.append("      }")
        out.extend(self._words_tail(fcols, word_filter, mode, U, stage, body))
        out.append("    }")
        if dense:
            out.append("    }")
        if full:
            out.append("    }")
        if mode == D.M_PART:
            out.append("    if (lane == 0) pend[cpos] = cbase + woff;")
        for s in cslots:  # unpack the chunk's 8-bit fields
            out.append("    " + " ".join(f"cn{s}_{g} += (uint32_t)(pc{s} >> {8 * g}) & 0xffu;" for g in range(G)) +
                       f" pc{s} = 0;")
        out.append("  }")
        for s in cslots:  # wave totals into lane 0's accumulator copy
            for g in range(G):
                out.append(f"  {{ uint32_t v_ = cn{s}_{g};")
                out.append("    for (int o = 32; o > 0; o >>= 1) v_ += (uint32_t)__shfl_xor((int)v_, o);")
                out.append(f"    if (lane == 0 && v_) acc_update<{D.S_SUM_I}>(acc + ({g} * {NS} + {s}) * {NCT} + copy, "
                           "(int64_t)v_); }")
        if mode == D.M_DENSE_LDS:
            out.append("  __syncthreads();")
            out.append(f"  const int flush_n = (int)d->G * {NS};")
            out.append(f"  for (int i = threadIdx.x; i < flush_n; i += {W * 64}) {{")
            out.append(f"    const int s = i % {NS};")
            ops = ", ".join(str(op) for op, _ in p.slots)
            inits = ", ".join(_lit(init) for _, init in p.slots)
            out.append(f"    constexpr int ops[{NS}] = {{{ops}}};")
            out.append(f"    constexpr int64_t init[{NS}] = {{{inits}}};")
            out.append(f"    const uint64_t* a = acc + (int64_t)i * {NCT};")
            out.append("    int64_t v = (int64_t)a[0];")
            out.append(f"    for (int k = 1; k < {NCT}; ++k) {{")
            out.append("      const int64_t x = (int64_t)a[k];")
            out.append("      switch (ops[s]) {")
            out.append(f"        case {D.S_SUM_I}: v += x; break;")
            out.append(f"        case {D.S_SUM_F}: v = __double_as_longlong(__longlong_as_double(v) + __longlong_as_double(x)); break;")
            out.append(f"        case {D.S_MIN_I}: v = x < v ? x : v; break;")
            out.append("        default: v = x > v ? x : v; break;")
            out.append("      }")
            out.append("    }")
            out.append("    if (v != init[s]) acc_update_rt(gacc + i, ops[s], v);")
            out.append("  }")
            if self.hll_lds and p.nhll:
                for ai, a in enumerate(p.aops):
                    if a["kind"] not in D.HLL_KINDS:
                        continue
                    # four byte registers per dword: one read (and rarely a CAS) per 4 registers
                    out.append(f"  {{ uint32_t* g = (uint32_t*)d->aops[{ai}].hll_regs;")
                    out.append(f"    const uint32_t* r = (const uint32_t*)hll{ai};")
                    out.append(f"    for (int i = threadIdx.x; i < (int)d->G * {self.m // 4}; i += {W * 64}) "
                               "hll_merge_word8(g + i, r[i]);")
                    out.append("  }")
        if mode == D.M_PART:
            out.append("  if (phout) {  // this block's level-1 histogram: column blockIdx.x of [part_n][gridDim.x]")
            out.append("    __syncthreads();")
            out.append(f"    for (int q = threadIdx.x; q <= (int)pmask; q += {W * 64}) "
                       "phout[(int64_t)q * gridDim.x + blockIdx.x] = phist[q];")
            out.append("  }")
        out.append("}")
        return "\n".join(out) + "\n"


_HDR_HASH: List[str] = []


def _hdr_hash() -> str:
    """Hash of the device headers the kernels include: a header change invalidates cached code."""
    if not _HDR_HASH:
        h = hashlib.sha256()
        for f in sorted(CSRC.glob("*.h")):
            h.update(f.read_bytes())
        _HDR_HASH.append(h.hexdigest())
    return _HDR_HASH[0]


def _code_key(src: str) -> str:
    return hashlib.sha256((src + "\0".join(OPTS) + _hdr_hash()).encode()).hexdigest()[:24]


_code_inflight: Dict[str, "Future"] = {}


def compile_code(src: str, name: str) -> bytes:
    """hipRTC-compile for gfx950 (no GPU needed), disk-cached by source + header hash.  Concurrent
    requests for one source wait on the first one's compile (one hipRTC run, one cache write)."""
    from concurrent.futures import Future

    from . import native

    key = _code_key(src)
    path = cache_dir() / f"{key}.co"
    if path.exists():
        return path.read_bytes()
    with _lock:
        fut = _code_inflight.get(key)
        owner = fut is None
        if owner:
            fut = _code_inflight[key] = Future()
    if not owner:
        return fut.result()
    try:
        code = native.load().rtc_compile(src, name, OPTS)
        # (unique per process and thread: other processes may share the cache directory)
        tmp = path.with_suffix(f".tmp{os.getpid()}.{threading.get_ident()}")
        tmp.write_bytes(code)
        os.replace(tmp, path)
    except BaseException as e:
        with _lock:
            _code_inflight.pop(key, None)
        fut.set_exception(e)
        raise
    with _lock:
        _code_inflight.pop(key, None)
    fut.set_result(code)
    return code


_inflight: Dict[str, "Future"] = {}
COMPILE_STATS = {"compiles": 0, "waits": 0}


def compile_source(src: str, name: str) -> int:
    """Compile (cached) and load into the current HIP context; returns a launch handle.

    ``_lock`` only guards the handle table: the compile itself (hipRTC, GIL released in the native
    binding) runs outside it, so different shapes compile in parallel and never stall a thread that
    only launches.  One future per source key: concurrent requests for the same shape wait on the
    first one's compile instead of compiling it again."""
    from concurrent.futures import Future

    from . import native

    key = _code_key(src)
    with _lock:
        h = _handles.get(key)
        if h is not None:
            return h
        fut = _inflight.get(key)
        owner = fut is None
        if owner:
            fut = _inflight[key] = Future()
    if not owner:
        COMPILE_STATS["waits"] += 1
        return fut.result()
    try:
        code = compile_code(src, name)
        h = native.load().module_load(code, name)
    except BaseException as e:
        with _lock:
            _inflight.pop(key, None)
        fut.set_exception(e)
        raise
    with _lock:
        _handles[key] = h
        _inflight.pop(key, None)
    COMPILE_STATS["compiles"] += 1
    fut.set_result(h)
    return h


def is_loaded(src: str) -> bool:
    """This source's kernel is compiled and loaded (no compile would run)."""
    return _code_key(src) in _handles


def kernel_meta(code: bytes) -> dict:
    """The AMDGPU metadata of a code object's first kernel (ELF note NT_AMDGPU_METADATA, msgpack):
    VGPR / SGPR counts and spills, private (scratch) and group segment sizes.  {} if absent."""
    import struct

    try:
        shoff = struct.unpack_from("<Q", code, 0x28)[0]
        shentsize, shnum = struct.unpack_from("<HH", code, 0x3A)
        for i in range(shnum):
            off = shoff + i * shentsize
            if struct.unpack_from("<I", code, off + 4)[0] != 7:  # SHT_NOTE
                continue
            so, ss = struct.unpack_from("<QQ", code, off + 0x18)
            p = so
            while p + 12 <= so + ss:
                nsz, dsz, typ = struct.unpack_from("<III", code, p)
                p += 12 + ((nsz + 3) & ~3)
                desc = code[p:p + dsz]
                p += (dsz + 3) & ~3
                if typ == 32:  # NT_AMDGPU_METADATA
                    import msgpack

                    md = msgpack.unpackb(desc, raw=False, strict_map_key=False)
                    ks = md.get("amdhsa.kernels") or [{}]
                    out = dict(ks[0])
                    out["amdhsa.target"] = md.get("amdhsa.target")
                    return out
    except (struct.error, ValueError, IndexError, ImportError):
        pass
    return {}


SGPR_SPILL_MAX = 128


class JitSpill(RuntimeError):
    """The kernel would spill registers to scratch (engine/device_exec.py _jit_build then tries a
    smaller unroll): a spilling scan is slow, and its scratch is allocated by the HIP runtime outside
    the torch allocator -- under memory pressure that allocation fails and aborts the queue."""


class NotCached(RuntimeError):
    """(``cached_only``) the kernel is not compiled yet; ``key`` names its code-cache entry."""

    def __init__(self, key: str):
        super().__init__(key)
        self.key = key


def is_cached(src: str) -> bool:
    key = _code_key(src)
    return key in _handles or (cache_dir() / f"{key}.co").exists()


class JitScan:
    """A compiled, specialized scan kernel for one ScanProgram shape."""

    def __init__(self, prog, mode: int, U: int, hll_lds: bool, m: int, narrow4: bool, load: bool = True,
                 budget: int = 150 * 1024, regstage: bool = False, shared: bool = False, literals: bool = False,
                 reject_spills: bool = False, cached_only: bool = False):
        self.literals = literals
        self._args = (prog, mode, U, hll_lds, m, narrow4, load, budget, regstage, shared)
        self.lay = layout(prog, mode, U, hll_lds, m, budget, regstage, shared)
        if self.lay.total > 160 * 1024:
            raise ValueError(f"jit layout needs {self.lay.total} B of LDS")
        g = _Gen(prog, mode, U, hll_lds, narrow4, self.lay, m, literals)
        tag = hashlib.sha1(repr((mode, U, self.lay.ncopy, regstage, self.lay.shared)).encode()
                           ).hexdigest()[:6]
        self.name = f"sdo_jit_{tag}"
        self.src = g.source(self.name)
        if cached_only and not is_cached(self.src):
            raise NotCached(_code_key(self.src))
        self.meta = kernel_meta(compile_code(self.src, self.name) or b"")
        # SGPR spills go to VGPR lanes (no scratch), but a few hundred of them turn the word loop into
        # writelane / readlane traffic: an unrolled count over one key spilled 1435 SGPRs at U=16,
        # 185 VALU per word instead of 13 at U=8 (profiles/r4/scan_kernel_ab_notes.md)
        self.spills = bool(self.meta.get(".private_segment_fixed_size") or self.meta.get(".vgpr_spill_count")
                           or int(self.meta.get(".sgpr_spill_count") or 0) > SGPR_SPILL_MAX)
        if self.spills and reject_spills:
            raise JitSpill(f"{self.name} U={U}: {self.meta.get('.vgpr_spill_count')} VGPR / "
                           f"{self.meta.get('.sgpr_spill_count')} SGPR spills, "
                           f"{self.meta.get('.private_segment_fixed_size')} B scratch")
        self.handle = compile_source(self.src, self.name) if load else -1
        self.U = U

    def specialized(self) -> "JitScan":
        """The same kernel with this program's query constants baked in as literals (a repeated
        statement's own code object: folded bounds, no descriptor loads, fewer live scalars --
        TPC-H Q19 3.4 vs 3.8 ms).  Same layout, grid and descriptor, so it swaps in place."""
        prog, mode, U, hll_lds, m, narrow4, load, budget, regstage, shared = self._args
        js = JitScan(prog, mode, U, hll_lds, m, narrow4, load, budget=budget, regstage=regstage,
                     shared=shared, literals=True)
        # literals can free or cost registers; a specialization that spills where the shape kernel
        # does not would be slower than the kernel it replaces
        return self if js.spills and not self.spills else js

    def occupancy(self) -> int:
        """Resident 512-thread workgroups per CU of the compiled kernel (registers and LDS)."""
        occ = self.__dict__.get("_occ")
        if occ is None:
            from . import native

            occ = self._occ = max(1, int(native.load().module_occupancy(self.handle, W * 64, int(self.lay.total))))
        return occ

    def launch(self, desc: torch.Tensor, grid: int) -> None:
        from . import native

        native.load().module_launch(self.handle, desc.data_ptr(), int(grid), W * 64, int(self.lay.total),
                                    native._stream(desc.device))
