"""Plain-PyTorch executor of a ``ScanProgram`` -- the CPU backend and the numerics oracle for the
HIP scan kernel (tests compare the two on the same shard).

It evaluates the same normalized filter IR, group keys, accumulator slots and HLL hashing as
``ops/csrc/olap_scan.hip`` with vectorized torch ops (no interpretation per row), producing the
same partial structures (dense ``[G, nslots]`` or sparse keys + accumulators).
"""
from __future__ import annotations

import os

import math
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import desc as D

_C1 = 0xFF51AFD7ED558CCD - (1 << 64)
_C2 = 0xC4CEB9FE1A85EC53 - (1 << 64)


def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:
    """logical shift right of int64 bit patterns"""
    if s == 0:
        return x
    return (x >> s) & ((1 << (64 - s)) - 1)


def mix64(x: torch.Tensor) -> torch.Tensor:
    x = x ^ _lsr(x, 33)
    x = x * _C1
    x = x ^ _lsr(x, 33)
    x = x * _C2
    x = x ^ _lsr(x, 33)
    return x


def clz64(x: torch.Tensor) -> torch.Tensor:
    n = torch.zeros_like(x)
    for s in (32, 16, 8, 4, 2, 1):
        top = _lsr(x, 64 - s) == 0
        n = torch.where(top, n + s, n)
        x = torch.where(top, x << s, x)
    return n


def fmix32(x: torch.Tensor) -> torch.Tensor:
    """murmur3 finalizer on uint32 values held in int64."""
    m = 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & m
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & m
    return x ^ (x >> 16)


def hll_update_values(vals: torch.Tensor, salt: int, p: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(bucket, rho) per value, bit-identical to ``hll_bucket_rho`` in csrc/sdo_device.h: values in
    [0, 2^32) use the 32-bit mix, others the 64-bit one."""
    v = vals.to(torch.int64)
    salt = int(salt)
    small = (v >= 0) & (v < (1 << 32))
    s32 = (salt ^ (salt >> 32)) & 0xFFFFFFFF
    h32 = fmix32((v & 0xFFFFFFFF) ^ s32)
    b32 = h32 >> (32 - p)
    rest32 = ((h32 << p) & 0xFFFFFFFF) | (1 << (p - 1))
    rho32 = clz64(rest32) - 32 + 1
    salt64 = salt - (1 << 64) if salt >= (1 << 63) else salt
    h = mix64(v ^ salt64)
    b64 = _lsr(h, 64 - p)
    rest = (h << p) | (1 << (p - 1))
    rho64 = clz64(rest) + 1
    return torch.where(small, b32, b64), torch.where(small, rho32, rho64)


def hll_estimate_torch(regs: torch.Tensor, p: int) -> torch.Tensor:
    """regs [G, m] int -> estimates [G] float64 (same formula as hll_estimate_kernel)."""
    m = float(1 << p)
    r = regs.to(torch.float64)
    s = torch.pow(2.0, -r).sum(dim=1)
    zeros = (regs == 0).sum(dim=1).to(torch.float64)
    alpha = 0.7213 / (1.0 + 1.079 / m)
    e = alpha * m * m / s
    lin = m * torch.log(m / torch.clamp(zeros, min=1.0))
    return torch.where((e <= 2.5 * m) & (zeros > 0), lin, e)


def _col(prog, name: str) -> torch.Tensor:
    from ..engine.lower import column_tensor

    return column_tensor(prog.ds, name)


def _rows(prog) -> torch.Tensor:
    parts = [torch.arange(a, b, dtype=torch.int64, device=prog.ds.device) for a, b in prog.ranges]
    return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=prog.ds.device)


def eval_bexpr(prog, x, rows: torch.Tensor) -> torch.Tensor:
    k = x[0]
    n = rows.numel()
    dev = rows.device
    if k == "true":
        return torch.ones(n, dtype=torch.bool, device=dev)
    if k == "false":
        return torch.zeros(n, dtype=torch.bool, device=dev)
    if k == "and":
        out = torch.ones(n, dtype=torch.bool, device=dev)
        for c in x[1]:
            out &= eval_bexpr(prog, c, rows)
        return out
    if k == "or":
        out = torch.zeros(n, dtype=torch.bool, device=dev)
        for c in x[1]:
            out |= eval_bexpr(prog, c, rows)
        return out
    if k == "not":
        return ~eval_bexpr(prog, x[1], rows)
    if k == "ids":
        ids = _col(prog, x[1])[rows].to(torch.int64)
        m = torch.from_numpy(np.ascontiguousarray(x[2])).to(dev)
        return m[ids]
    if k == "time":
        u = prog.ds.time_unit_ms
        t = prog.ds.time[rows].to(torch.int64)
        lo = -(-x[1] // u)
        hi = -(-x[2] // u)
        return (t >= lo) & (t < hi)
    if k == "timeset":
        t = prog.ds.time[rows].to(torch.int64)
        allowed = torch.from_numpy(np.asarray(x[1], dtype=np.int64)).to(dev)
        return torch.isin(t, allowed)
    if k == "int":
        v = _col(prog, x[1])[rows].to(torch.int64)
        return (v >= x[2]) & (v <= x[3])
    if k == "flt":
        v = _col(prog, x[1])[rows].to(torch.float64)
        lo_ok = v > x[2] if x[4] & 1 else v >= x[2]
        hi_ok = v < x[3] if x[4] & 2 else v <= x[3]
        return lo_ok & hi_ok
    if k == "fexpr":
        v = _ast_values(prog, x[1], rows)
        lo_ok = v > x[2] if x[4] & 1 else v >= x[2]
        hi_ok = v < x[3] if x[4] & 2 else v <= x[3]
        return lo_ok & hi_ok
    raise ValueError(k)


def _ast_values(prog, n, rows: torch.Tensor) -> torch.Tensor:
    """f64 value per row of an expression AST (expression filters; same value model as the
    device VM: metrics with decimal scale, dimensions through their f64 dictionary table)."""
    from ..engine.lower import dim_numeric_lut

    k = n[0]
    if k == "const":
        return torch.full((rows.numel(),), float(n[1]), dtype=torch.float64, device=rows.device)
    if k == "lut":
        ids = _col(prog, n[1])[rows].to(torch.int64)
        return n[2].to(rows.device)[ids]
    if k == "col":
        name = n[1]
        ds = prog.ds
        if name in ds.dims:
            ids = _col(prog, name)[rows].to(torch.int64)
            return dim_numeric_lut(ds, name).to(rows.device)[ids]
        if name == "__time":
            return ds.time[rows].to(torch.float64) * float(ds.time_unit_ms)
        v = _col(prog, name)[rows].to(torch.float64)
        m = ds.metrics.get(name)
        if m is not None and m.kind == "decimal" and m.scale:
            v = v * (10.0 ** -m.scale)
        return v
    if k in ("neg", "abs", "floor", "ceil", "sqrt", "log", "exp"):
        a = _ast_values(prog, n[1], rows)
        return {"neg": torch.neg, "abs": torch.abs, "floor": torch.floor, "ceil": torch.ceil, "sqrt": torch.sqrt,
                "log": torch.log, "exp": torch.exp}[k](a)
    a, b = _ast_values(prog, n[1], rows), _ast_values(prog, n[2], rows)
    if k == "pmod":
        m = torch.fmod(a, b)
        return torch.where(m < 0, torch.fmod(m + b, b), m)
    return {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div, "min": torch.minimum,
            "max": torch.maximum, "mod": torch.fmod, "pow": torch.pow}[k](a, b)


def _time_field(ms: torch.Tensor, kc) -> torch.Tensor:
    from ..query import granularity as Gr

    tf = kc.tfield
    ms = ms + kc.tz_ms
    fd = lambda a, b: torch.div(a, b, rounding_mode="floor")  # noqa: E731
    if tf == Gr.T_MS:
        return ms
    if tf == Gr.T_SECOND:
        return fd(ms, 1000)
    if tf == Gr.T_MINUTE:
        return fd(ms, 60_000)
    if tf == Gr.T_HOUR:
        return fd(ms, 3_600_000)
    if tf == Gr.T_DAY:
        return fd(ms, 86_400_000)
    if tf == Gr.T_WEEK:
        return fd(fd(ms, 86_400_000) + 3, 7)
    if tf == Gr.T_PERIOD:
        return fd(ms - kc.origin_ms, kc.period_ms)
    if tf == Gr.T_HOD:
        return fd(ms, 3_600_000) - fd(ms, 86_400_000) * 24
    if tf == Gr.T_MOH:
        return fd(ms, 60_000) - fd(ms, 3_600_000) * 60
    if tf == Gr.T_SOM:
        return fd(ms, 1000) - fd(ms, 60_000) * 60
    days = fd(ms, 86_400_000)
    if tf == Gr.T_DOW:
        return torch.remainder(days + 3, 7) + 1
    z = days + 719468
    era = fd(z, 146097)
    doe = z - era * 146097
    yoe = torch.div(doe - torch.div(doe, 1460, rounding_mode="trunc") + torch.div(doe, 36524, rounding_mode="trunc")
                    - torch.div(doe, 146096, rounding_mode="trunc"), 365, rounding_mode="trunc")
    y = yoe + era * 400
    doy = doe - (365 * yoe + torch.div(yoe, 4, rounding_mode="trunc") - torch.div(yoe, 100, rounding_mode="trunc"))
    mp = torch.div(5 * doy + 2, 153, rounding_mode="trunc")
    d = doy - torch.div(153 * mp + 2, 5, rounding_mode="trunc") + 1
    m = torch.where(mp < 10, mp + 3, mp - 9)
    y = y + (m <= 2).to(torch.int64)
    if tf == Gr.T_MONTH:
        return y * 12 + (m - 1)
    if tf == Gr.T_QUARTER:
        return y * 4 + torch.div(m - 1, 3, rounding_mode="trunc")
    if tf == Gr.T_YEAR:
        return y
    if tf == Gr.T_MOY:
        return m
    if tf == Gr.T_DOM:
        return d
    if tf == Gr.T_QOY:
        return torch.div(m - 1, 3, rounding_mode="trunc") + 1
    if tf == Gr.T_DOY:
        from ..query.intervals import days_from_civil

        yy = y.cpu().numpy()
        jan1 = torch.from_numpy(np.array([days_from_civil(int(a), 1, 1) for a in yy], dtype=np.int64)).to(ms.device)
        return days - jan1 + 1
    raise ValueError(tf)


def compute_keys(prog, rows: torch.Tensor) -> torch.Tensor:
    key = torch.zeros(rows.numel(), dtype=torch.int64, device=rows.device)
    for kc in prog.keys:
        v = _col(prog, kc.col)[rows].to(torch.int64)
        if kc.kind == D.K_REMAP:
            rm = torch.from_numpy(kc.remap.astype(np.int64)).to(rows.device)
            v = rm[v]
        elif kc.kind == D.K_TIME:
            v = _time_field(v * prog.ds.time_unit_ms, kc) - kc.base
            v = v.clamp(0, kc.card - 1)
        elif kc.kind == D.K_INT:
            v = (v - kc.base).clamp(0, kc.card - 1)
        elif kc.base:
            v = v - kc.base  # K_ID in a shard-local key window
        key += v * kc.stride
    return key


def _expr_values(prog, eops, rows: torch.Tensor) -> torch.Tensor:
    st: List[torch.Tensor] = []
    for op, col, c in eops:
        if op == D.E_LUT:
            ids = _col(prog, prog.colname(col))[rows].to(torch.int64)
            lut = prog.lut_ptrs.get(c)
            if lut is None:
                lut = prog.luts[prog.colname(col)]
            st.append(lut.to(rows.device)[ids])
        elif op == D.E_COL:
            v = _col(prog, prog.colname(col))[rows].to(torch.float64)
            st.append(v * c if c != 0.0 else v)
        elif op == D.E_CONST:
            st.append(torch.full((rows.numel(),), c, dtype=torch.float64, device=rows.device))
        elif op == D.E_NEG:
            st[-1] = -st[-1]
        elif op == D.E_ABS:
            st[-1] = st[-1].abs()
        elif op in (D.E_FLOOR, D.E_CEIL, D.E_SQRT, D.E_LOG, D.E_EXP):
            st[-1] = {D.E_FLOOR: torch.floor, D.E_CEIL: torch.ceil, D.E_SQRT: torch.sqrt, D.E_LOG: torch.log,
                      D.E_EXP: torch.exp}[op](st[-1])
        elif op in (D.E_MOD, D.E_PMOD, D.E_POW):
            b = st.pop()
            a = st.pop()
            if op == D.E_POW:
                st.append(torch.pow(a, b))
            else:
                m = torch.fmod(a, b)
                if op == D.E_PMOD:
                    m = torch.where(m < 0, torch.fmod(m + b, b), m)
                st.append(m)
        else:
            b = st.pop()
            a = st.pop()
            st.append({D.E_ADD: a + b, D.E_SUB: a - b, D.E_MUL: a * b, D.E_DIV: a / b,
                       D.E_MIN: torch.minimum(a, b), D.E_MAX: torch.maximum(a, b)}[op])
    return st[-1]


def _agg_values(prog, a, rows: torch.Tensor) -> torch.Tensor:
    """int64 payload per row for an aggregator (float kinds: f64 bits / ordered ints)."""
    k = a["kind"]
    if k == D.A_COUNT:
        return torch.ones(rows.numel(), dtype=torch.int64, device=rows.device)
    if k == D.A_SUM_X:
        return torch.round(_expr_values(prog, a["expr"], rows)).to(torch.int64)
    if k in (D.A_SUM_F, D.A_MIN_F, D.A_MAX_F):
        if a.get("expr"):
            f = _expr_values(prog, a["expr"], rows)
        else:
            f = _col(prog, prog.colname(a["col"]))[rows].to(torch.float64)
        if k == D.A_SUM_F:
            return f
        b = f.view(torch.int64)
        return torch.where(b >= 0, b, b ^ 0x7FFFFFFFFFFFFFFF)
    v = _col(prog, prog.colname(a["col"]))[rows]
    if v.dtype.is_floating_point:
        v = v.to(torch.float64).trunc()
    return v.to(torch.int64)


def run_reference(prog, sparse: Optional[bool] = None):
    """Execute a program with torch.  Returns (kind, keys, acc, hll_list)."""
    from ..engine.partials import Partials

    ds = prog.ds
    dev = ds.device
    m = 1 << prog.hll_p
    nslots = prog.nslots
    if sparse is None:
        sparse = prog.G > int(os.environ.get("SDO_REF_SPARSE_G", 1 << 22))
    rows = _rows(prog) if not prog.empty else torch.zeros(0, dtype=torch.int64, device=dev)
    mask = eval_bexpr(prog, prog.bexpr, rows) if rows.numel() else torch.zeros(0, dtype=torch.bool, device=dev)
    rows = rows[mask]
    key = compute_keys(prog, rows)
    if sparse:
        uk, inv = torch.unique(key, return_inverse=True)
        R = uk.numel()
        idx = inv
    else:
        R = prog.G
        idx = key
    acc = torch.empty((R, nslots), dtype=torch.int64, device=dev)
    for s, (op, init) in enumerate(prog.slots):
        acc[:, s] = init
    for a in prog.aops:
        if a["kind"] in (D.A_HLL, D.A_HLL_CODE, D.A_HLL_STORED, D.A_ROWID):
            continue
        amask = torch.ones(rows.numel(), dtype=torch.bool, device=dev)
        if a.get("filter") is not None:
            amask = eval_bexpr(prog, a["filter"], rows)
        r, ix = rows[amask], idx[amask]
        vals = _agg_values(prog, a, r)
        s = a["slot"]
        op = prog.slots[s][0]
        col = acc[:, s].clone()
        if op == D.S_SUM_I:
            col.index_add_(0, ix, vals)
        elif op == D.S_SUM_F:
            cf = col.view(torch.float64).clone()
            cf.index_add_(0, ix, vals)
            col = cf.view(torch.int64)
        elif op == D.S_MIN_I:
            col.scatter_reduce_(0, ix, vals, reduce="amin", include_self=True)
        else:
            col.scatter_reduce_(0, ix, vals, reduce="amax", include_self=True)
        acc[:, s] = col
    hlls = []
    for a in prog.aops:
        if a["kind"] not in D.HLL_KINDS:
            continue
        amask = torch.ones(rows.numel(), dtype=torch.bool, device=dev)
        if a.get("filter") is not None:
            amask = eval_bexpr(prog, a["filter"], rows)
        r, ix = rows[amask], idx[amask]
        c = _col(prog, prog.colname(a["col"]))
        if a["kind"] == D.A_HLL_CODE:  # u16 bucket << 5 | rho (segment/hllcode.py)
            code = c.view(torch.int16)[r].to(torch.int64) & 0xFFFF
            bucket, rho = code >> 5, code & 31
        else:
            bucket, rho = hll_update_values(c[r].to(torch.int64), a.get("salt", 0), prog.hll_p)
        regs = torch.zeros(R * m, dtype=torch.int64, device=dev)
        regs.scatter_reduce_(0, ix * m + bucket, rho, reduce="amax", include_self=True)
        hlls.append(regs.view(R, m).to(torch.uint8))  # byte registers, like the scan kernels
    if sparse:
        return Partials("sparse", acc, uk, hlls)
    return Partials("dense", acc, None, hlls)


def run_reference_mask(prog) -> torch.Tensor:
    """Row ids passing the filter (select queries)."""
    dev = prog.ds.device
    if prog.empty:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    rows = _rows(prog)
    return rows[eval_bexpr(prog, prog.bexpr, rows)]
