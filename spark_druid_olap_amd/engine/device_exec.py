"""Run a ScanProgram on the GPU with the HIP kernel (``ops/csrc/olap_scan.hip``).

``PreparedScan`` owns the device buffers (descriptor, accumulators, HLL registers, hash table)
so a prepared query re-executes with a handful of fills + ONE kernel launch -- the descriptor is
uploaded once at prepare time, pointers are stable across runs.

Mode choice (per shard): accumulators + HLL registers that fit the LDS budget run fully in LDS
(flushed once per workgroup); larger dense key spaces accumulate with global atomics; key spaces
too large for a dense array use the global open-addressing hash table, sized from the cost
model's row estimate and grown on overflow.
"""
from __future__ import annotations

import contextlib
import math
import os
import threading
import weakref
from collections import OrderedDict
from typing import List, Optional

import numpy as np
import torch

from ..ops import desc as D
from ..ops import native
from .lower import ScanProgram, pack
from .partials import Partials
from .scheduler import current_slot

from ..planner.cost import PLAN_LDS_BUDGET as LDS_BUDGET  # noqa: E402  (single source: the cost model)
# one accumulator table per workgroup (JIT only) for key spaces whose per-wave copies do not fit:
# up to this many bytes of LDS, instead of HBM atomics contending on the touched groups
from ..planner.cost import SHARED_LDS_MAX  # noqa: E402,F401
BLOCK = 512
UNROLL = 2  # (interpreter kernel: words per step)
BLOCKS_PER_CU = 3
USE_JIT = os.environ.get("SDO_JIT", "1") != "0"
JIT_BLOCKS = 3       # target resident workgroups per CU
JIT_STAGE = "auto"   # auto | reg (VGPR loads) | lds (LDS-DMA planes)
JIT_TRACE = False    # (tools: print the unroll / budget candidates tried)
FORCE_U = 0  # cap the words per step of generated kernels (0: the register / LDS-driven choice)
# Literal specialization of repeated statements (ops/jit.py JitScan.specialized): a prepared scan's
# first runs use the shape's shared kernel (query constants read from the descriptor: every
# parameterization of a dashboard query shares one code object); from its SPECIALIZE_AFTER-th run
# a kernel with the constants baked in is compiled -- in the background ("async": serving never
# waits for hipRTC) or at once ("sync": a benchmark's warmup) -- and swapped in.
# A background compile costs ~0.3-1 s of a host core (hipRTC, GIL released) and saves a few to tens
# of microseconds per run, so only statements that keep coming back are worth it: at most
# SPEC_MAX_PENDING compiles queue at once, and a statement that finds the queue full asks again
# after twice as many runs (a dashboard's hot statements get there; 2,000 one-off
# parameterizations do not flood the host with compiles).
SPECIALIZE = os.environ.get("SDO_JIT_SPECIALIZE", "async")  # off | async | sync
SPECIALIZE_AFTER = int(os.environ.get("SDO_JIT_SPECIALIZE_AFTER", "4"))
SPEC_MAX_PENDING = 2
_spec_pending = [0]
_spec_lock = threading.Lock()
_spec_pool = []


def _spec_executor():
    if not _spec_pool:
        from concurrent.futures import ThreadPoolExecutor

        _spec_pool.append(ThreadPoolExecutor(max_workers=SPEC_MAX_PENDING, thread_name_prefix="sdo-jit-spec"))
    return _spec_pool[0]


def _spec_job(js):
    from ..utils.metrics import count_event

    try:
        return js.specialized()
    finally:
        count_event("jit_spec_done")
        with _spec_lock:
            _spec_pending[0] -= 1


# The packed layout pays off where a scan streams: whole-chunk walks over LDS tables.  A selective
# scan mostly walks single nonzero words (two stream loads per packed column and word vs one plain
# load): TPC-H Q5 (2.5% of rows) 0.25 -> 0.18 ms packed, Q7 (0.3%) 0.37 -> 0.50 ms.  Scans bound
# by random accesses -- id-set filter probes, HBM-table atomics -- lose occupancy to the unrolled
# runs and gain nothing: TPC-H22 Q9 (p_name id set) 4.95 -> 5.49 ms, Q11 (HBM table) 3.61 ->
# 4.18 ms packed (profiles/r4/scan_kernel_ab_notes.md).
PACKED_MODES = (D.M_DENSE_LDS,)
PACK_MIN_SELECTIVITY = 0.02


def _attach_packed(prog, mode: int) -> None:
    """Bit-packed copies (segment/packed.py) of the integer columns the program reads: the JIT
    kernel reads those instead of the byte-wide columns (the interpreter never does).  Only the
    table-aggregating modes walk whole chunks in the static runs the layout is built for; the
    partition / emit producers keep the plain columns."""
    from ..segment import packed as PK

    prog.packed = {}
    if not PK.ENABLED or prog.empty or prog.ds.device.type != "cuda" or mode not in PACKED_MODES:
        return
    n = max(1, int(prog.ds.num_rows))
    if float(getattr(prog, "est_rows", n)) < PACK_MIN_SELECTIVITY * n:
        return
    if any(int(f[0]) == D.F_IN_SET for f in prog.fops):
        return
    for name in list(prog.fcols) + list(prog.pcols):
        pc = PK.packed_column(prog.ds, name)
        if pc is not None:
            prog.packed[name] = pc


def _jit_for(prog, mode: int, hll_lds: bool, m: int, shared: bool = False):
    """Specialized kernel for this program shape (None -> use the interpreter, plain columns)."""
    if not USE_JIT:
        prog.packed = {}
        return None
    from ..ops import jit

    if getattr(prog, "packed", None) is None:
        _attach_packed(prog, mode)
    js = _jit_build(prog, mode, hll_lds, m, shared)
    if js is None:
        prog.packed = {}  # the interpreter reads the plain columns
    return js


# First-seen shapes while serving (server/gateway.py: ``with async_compile():`` around a statement's
# prepare).  A new kernel shape costs a hipRTC compile of ~0.3 s alone and 1-2 s on a host busy
# with 64 clients -- the BI plan's cold p99 (profiles/r5/thrift_jmx_s8_sf100_c64_cold_*.json).  In
# the scope, a scan whose kernel is not compiled yet runs on the interpreter kernel (ops/csrc, same
# results, a few times slower) while the JIT source compiles on a background thread; the session
# re-prepares the statement once every compile it started has finished (session.py
# prepare_druid), and the next execution runs the JIT kernel from the code cache.  Only plans the
# interpreter runs as-is take the detour: per-wave LDS copies, plain HBM tables, hash tables, masks
# -- shared LDS tables, first-touch / presence byte tables and the partitioned producers would fall
# back to other modes (a 150M-group HBM table per slot), so those still compile in the foreground.
# Round 5 turned this off after the BI plan under 64 clients faulted (illegal address) with it on.
# Both suspects were checked on the GPU (tests/test_gpu_bi_templates.py): the interpreter kernel
# answers every BI template correctly, alone and as the interim plan.  What the detour changed is
# WHEN plans are built: a re-prepare swaps a new plan in while other slots run, and the device
# artifacts its lowering builds lazily -- bit-packed column copies, HLL code planes, FD tables --
# were published to datasource-wide caches while their producing kernels were still queued on the
# preparing thread's stream; a slot whose stream was ordered after the default stream at lease
# time, earlier, could then scan a half-written column (garbage ids -> out-of-bounds table
# indices).  Every such cache now publishes only completed artifacts (utils/streams.py), and a
# fresh plan is published after its prepare's stream drained (session.py prepare_druid).
ASYNC_JIT = os.environ.get("SDO_ASYNC_JIT", "1") == "1"
ASYNC_JIT_WORKERS = 4
_async_tls = threading.local()
_async_failed: set = set()
_async_pool: list = []
_async_futs: list = []  # background compiles not known to be finished (wait_background_compiles)


def wait_background_compiles(timeout: float = 120.0) -> int:
    """Block until the first-seen-shape compiles started so far have finished (a server's warm-up:
    the interim plans they belong to re-prepare at their next run); returns how many were waited
    for."""
    import concurrent.futures as cf

    with _spec_lock:
        futs = [f for f in _async_futs if not f.done()]
    if futs:
        cf.wait(futs, timeout=timeout)
    return len(futs)


@contextlib.contextmanager
def async_compile():
    """Scope in which prepares start first-seen kernel compiles in the background (see above)."""
    prev = getattr(_async_tls, "pending", None)
    _async_tls.pending = [] if ASYNC_JIT and USE_JIT else None
    try:
        yield
    finally:
        _async_tls.pending = prev


def prepare_collecting(fn):
    """``fn()`` and the background compiles it started (empty outside ``async_compile``)."""
    pend = getattr(_async_tls, "pending", None)
    if pend is None:
        return fn(), []
    n = len(pend)
    r = fn()
    return r, pend[n:]


def _async_ok(prog, mode: int, shared: bool) -> bool:
    return (mode in (D.M_DENSE_LDS, D.M_DENSE_GLOBAL, D.M_HASH, D.M_MASK) and not shared
            and not getattr(prog, "touch_table", False) and not getattr(prog, "presence_bytes", False))


def _async_job(prog, mode: int, hll_lds: bool, m: int, shared: bool, narrow4: bool, key: str):
    from ..utils.metrics import count_event

    try:
        _jit_select(prog, mode, hll_lds, m, shared, load=False, narrow4=narrow4)
    except BaseException:
        _async_failed.add(key)
        raise
    finally:
        count_event("jit_async_done")


def _jit_build(prog, mode: int, hll_lds: bool, m: int, shared: bool = False, load: bool = True):
    """(``load=False``: compile only -- tools/jit_isa.py inspects the exact kernel a scan would run
    on a host without a GPU.)"""
    from ..ops import jit

    pend = getattr(_async_tls, "pending", None)
    if load and pend is not None and _async_ok(prog, mode, shared):
        narrow4 = bool(native.narrow4())
        try:
            return _jit_select(prog, mode, hll_lds, m, shared, load=True, narrow4=narrow4, cached_only=True)
        except jit.NotCached as e:
            if e.key not in _async_failed:
                import copy

                if not _async_pool:
                    from concurrent.futures import ThreadPoolExecutor

                    _async_pool.append(ThreadPoolExecutor(max_workers=ASYNC_JIT_WORKERS,
                                                          thread_name_prefix="sdo-jit-async"))
                # (a snapshot: the prepare goes on to mark the program for the interpreter)
                snap = copy.copy(prog)
                fut = _async_pool[0].submit(_async_job, snap, mode, hll_lds, m, shared, narrow4, e.key)
                pend.append(fut)
                with _spec_lock:
                    _async_futs[:] = [f for f in _async_futs if not f.done()] + [fut]
                from ..utils.metrics import count_event

                count_event("jit_async_interim")
                return None
    return _jit_select(prog, mode, hll_lds, m, shared, load=load)


def _jit_select(prog, mode: int, hll_lds: bool, m: int, shared: bool = False, load: bool = True,
                narrow4: Optional[bool] = None, cached_only: bool = False):
    from ..ops import jit

    if narrow4 is None:
        narrow4 = bool(native.narrow4()) if load else True

    nplanes = sum(2 if column_tensor_size(prog, c) == 8 else 1 for c in prog.cols)
    prefs = [16, 8, 4, 2] if nplanes <= 3 else ([8, 4, 2] if nplanes <= 8 else [4, 2])
    if FORCE_U:  # (tools/query_probe.py A/B of the word unroll)
        prefs = [u for u in prefs if u <= FORCE_U] or [prefs[-1]]
    # occupancy first: the scan is latency-bound at 8 waves/CU, so prefer the largest U that still
    # leaves room for JIT_BLOCKS workgroups per CU (160 KiB LDS), then fall back to one workgroup
    budgets = [(160 * 1024) // b - 512 for b in (JIT_BLOCKS, 1) if b >= 1]
    regstage = JIT_STAGE == "reg" or (JIT_STAGE == "auto" and jit.prefer_regstage(prog))
    for budget in budgets:
        for U in prefs:
            lay = jit.layout(prog, mode, U, hll_lds, m, budget, regstage, shared)
            if JIT_TRACE:
                print(f"[jit] U={U} budget={budget} LDS={lay.total} ncopy={lay.ncopy}", flush=True)
            if lay.total <= budget and (shared or mode != D.M_DENSE_LDS or lay.ncopy >= 4 or U == prefs[-1]):
                try:
                    # a kernel that would spill registers takes the next smaller unroll
                    return jit.JitScan(prog, mode, U, hll_lds, m, narrow4,
                                       load=load, budget=budget, regstage=regstage, shared=shared,
                                       reject_spills=U != prefs[-1], cached_only=cached_only)
                except jit.JitSpill as e:
                    if JIT_TRACE:
                        print(f"[jit] U={U} budget={budget} rejected: {e}", flush=True)
                    continue
                except jit.NotCached:
                    raise
                except Exception as e:  # pragma: no cover - compile problems fall back loudly
                    import warnings

                    warnings.warn(f"JIT compile failed, using the interpreter kernel: {e}")
                    return None
    return None


def column_tensor_size(prog, name: str) -> int:
    from .lower import column_tensor

    return column_tensor(prog.ds, name).element_size()

_cu_cache = {}


def num_cus(dev: torch.device) -> int:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _cu_cache:
        _cu_cache[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count)
    return _cu_cache[idx]


def _next_pow2(x: int) -> int:
    return 1 << max(10, int(math.ceil(math.log2(max(2, x)))))


class PreparedScan:
    def __init__(self, prog: ScanProgram, mode: Optional[int] = None, dense_max: Optional[int] = None):
        self.prog = prog
        ds = prog.ds
        self.dev = ds.device
        self.m = 1 << prog.hll_p
        G, ns = prog.G, prog.nslots
        acc_bytes = G * ns * 8 * (BLOCK // 64)  # one private copy per wave
        hll_bytes = prog.nhll * G * self.m * 4
        self.hll_lds = 0
        self.shared = False
        shared_bytes = G * ns * 8
        # the cost model decides the group-by table (planner/cost.py plan_groupby): LDS copies /
        # shared LDS table / HBM table (with first-touch or presence byte tables) / hash table
        from ..planner.cost import plan_groupby

        self.plan = plan_groupby(prog, USE_JIT, dense_max is not None)
        if mode is None:
            mode = {"dense-lds": D.M_DENSE_LDS, "dense-global": D.M_DENSE_GLOBAL, "hash": D.M_HASH,
                    "partitioned": D.M_PART}[self.plan.mode]
            self.shared = self.plan.shared
            self.hll_lds = 1 if self.plan.hll_lds else 0
        self.mode = mode
        self.dedup = 1 if G <= 64 else 0
        if mode == D.M_DENSE_LDS:
            self.lds = (shared_bytes if self.shared else acc_bytes) + (hll_bytes if self.hll_lds else 0)
            self.lds = (self.lds + 15) // 16 * 16
        else:
            self.lds = 0
        if mode == D.M_HASH:
            est = max(1024, min(prog.G, int(prog.est_rows * 1.2) + 1024))
            self.cap = _next_pow2(2 * est)
        else:
            self.cap = 0
        self.jit = None
        self._runs = 0
        self._spec_at = SPECIALIZE_AFTER  # run count at which a literal-specialized kernel is asked for
        self._spec_future = None
        self.part = None
        self.part_having = None
        self.part_topk = None  # (k, slot, is_f64, desc): ORDER BY <aggregate> LIMIT k fused (set_part_topk)
        self.part_cap = 1 << 16
        if mode == D.M_PART and not prog.empty:
            # radix-partitioned group-by (ops/csrc/partition.hip): the JIT producer appends records
            self.jit = _jit_for(prog, D.M_PART, False, self.m)
            if self.jit is None:
                mode = D.M_DENSE_GLOBAL  # no JIT: the HBM table with atomics
            else:
                self.part = part_layout(prog)
        elif mode == D.M_PART:
            mode = D.M_DENSE_GLOBAL
        self.mode = mode
        # existence-only dense HBM scan on one GPU: one byte per group (150M order groups -> 150 MB,
        # which stays in the 256 MB Infinity Cache) instead of an 8-byte counter row
        self.pres_bytes = bool(mode == D.M_DENSE_GLOBAL and self.plan.presence_bytes)
        prog.presence_bytes = self.pres_bytes
        # large dense HBM table (TPC-H Q3: 150M order groups, ~1M touched): a first-touch byte per
        # group written by the scan; compaction reads G bytes instead of G x nslots x 8, and only
        # the touched rows are re-initialised after the run (no full-table fill per execution)
        self.touch = bool(mode == D.M_DENSE_GLOBAL and self.plan.touch and not self.pres_bytes)
        prog.touch_table = self.touch
        prog.hll32 = False
        if not prog.empty and mode != D.M_PART:
            # the JIT keeps LDS registers one byte each (hll_update8)
            jit_hll_lds = bool(prog.nhll) and mode == D.M_DENSE_LDS and hll_bytes // 4 <= LDS_BUDGET \
                and not self.shared
            # global registers: u32 atomics during the scan while the table is small (one atomicMax
            # per update instead of a byte CAS loop: SSB "HLL customers" 4.5 -> 2.9 ms), bytes after
            rows_ = self.cap if mode == D.M_HASH else G
            n_glob = prog.nhll_total - (prog.nhll if jit_hll_lds else 0)
            prog.hll32 = bool(n_glob) and n_glob * rows_ * self.m * 4 <= HLL32_MAX_BYTES and not jit_hll_lds
            self.jit = _jit_for(prog, mode, jit_hll_lds, self.m, self.shared)
            if self.pres_bytes and self.jit is None:
                self.pres_bytes = prog.presence_bytes = False
                self.jit = _jit_for(prog, mode, jit_hll_lds, self.m, self.shared)
            if self.touch and self.jit is None:
                self.touch = prog.touch_table = False
            if self.shared and self.jit is None:
                # the interpreter kernel only knows per-wave copies: accumulate in HBM instead
                self.mode, self.shared, self.lds = D.M_DENSE_GLOBAL, False, 0
                self.jit = _jit_for(prog, self.mode, False, self.m)
        # stored (rolled-up) HLL sketches: the JIT kernel unions them in the scan (A_HLL_STORED);
        # the interpreter leaves them to the executor (engine/executor.py _merge_stored_hll)
        # (partitioned: the records carry the row ids, part_agg unions the stored pairs per group)
        self.stored_fused = bool(prog.stored_hll) and self.jit is not None
        self.hll32 = bool(getattr(prog, "hll32", False)) and self.jit is not None
        prog.hll32 = self.hll32
        self._slot_lock = threading.Lock()
        self._slots = {}
        weakref.finalize(self, _forget_prep, id(self))
        self._settle()

    # ------------------------------------------------------------------ buffers
    # Every execution slot (engine/scheduler.py) gets its own accumulators / hash table / HLL
    # registers / descriptor, so concurrent runs of one prepared query on different streams never
    # share device state; the generated kernel, grid and mode are shared.  Leased slots carve the
    # large tensors from the slot's arena (SlotArena), slot 0 allocates them per scan.
    def _bufs(self) -> "_Bufs":
        slot = current_slot()
        b = self._slots.get(slot)
        if slot != 0:
            return self._arena_bufs(slot, b, self.cap)
        if b is None:
            # allocated without holding this scan's lock: an out-of-memory eviction takes the locks
            # of the scans it evicts, and two threads each holding their own scan's lock while
            # evicting the other's would deadlock
            nb = _with_eviction(lambda: self._alloc(self.cap), self, slot)
            with self._slot_lock:
                b = self._slots.get(slot)
                if b is None:
                    b = self._slots[slot] = nb
            _buffers_acquired(self, slot, b)
        else:
            _buffers_used(self, slot)
        return b

    def _rebuf(self, cap: int) -> "_Bufs":
        """This slot's buffers re-made for a new capacity (hash-table growth / adaptive size)."""
        slot = current_slot()
        if slot != 0:
            with self._slot_lock:
                self._slots.pop(slot, None)
            return self._arena_bufs(slot, None, cap)
        nb = self._slots[slot] = _with_eviction(lambda: self._alloc(cap), self, slot)
        _buffers_acquired(self, slot, nb)
        return nb

    def _tensor_layout(self, cap: int) -> list:
        """(name, elements, dtype, shape) of the large per-slot tensors, in carving order."""
        prog = self.prog
        rows = self._rows(cap)
        nblocks = prog.nhll_total if self.stored_fused else prog.nhll
        if self.pres_bytes:
            # padded to whole 8-byte words (the fused reset zeroes words; padding bytes stay 0
            # and never compact)
            items = [("acc", (rows + 7) // 8 * 8, torch.uint8, None)]
        else:
            items = [("acc", rows * prog.nslots, torch.int64, (rows, prog.nslots))]
        items.append(("keys", rows if self.mode == D.M_HASH else 1, torch.int64, None))
        # byte registers (sdo_device.h hll_update8 / hll_merge_word8): the partials, the wire and
        # the estimator all read u8; scan-time u32 registers (narrowed into them after each run)
        items += [("hll", rows * self.m, torch.uint8, None)] * nblocks
        if self.hll32:
            items += [("hll32", rows * self.m, torch.int32, None)] * nblocks
        # (padded to whole 64-group words: native.touch_compact reads it 16 bytes per lane)
        items.append(("touch", ((rows + 63) // 64 * 64) if self.touch else 64, torch.uint8, None))
        return items

    def _arena_bufs(self, slot: int, b: Optional["_Bufs"], cap: int) -> "_Bufs":
        from .scheduler import slot_epoch

        ar = slot_arena(self.dev, slot)
        ep = slot_epoch(slot)
        if b is not None and b.arena is not None and b.arena[0] == ar.gen and b.arena[2] == ep:
            return b  # already carved in this statement
        items = self._tensor_layout(cap)
        sizes = [n * torch.empty((), dtype=dt).element_size() for _, n, dt, _ in items]
        offs, total = _carve_aligned(sizes)
        gen, off, intact, buf = ar.carve(total, self)
        if b is not None and b.arena is not None and b.arena[:2] == (gen, off) and b.cap == cap:
            b.arena = (gen, off, ep)
            if not intact:
                b.clean = False  # another scan wrote over the region: the next launch resets it
            return b
        v = _Bufs()
        v.geom = self._geom(cap)
        v.hll, v.hll32 = [], []
        for (name, n, dt, shape), o in zip(items, offs):
            t = SlotArena.view(buf, off + o, n, dt, shape)
            if name in ("hll", "hll32"):
                getattr(v, name).append(t)
            else:
                setattr(v, name, t)
        v.overflow = torch.zeros(1, dtype=torch.int32, device=self.dev)
        nb = self._alloc(cap, v)
        nb.arena = (gen, off, ep)
        with self._slot_lock:
            self._slots[slot] = nb
        return nb

    def _settle(self) -> None:
        """The LDS-budget mode fallback, decided at prepare time without allocating: buffers are
        allocated per execution slot on first use (a server prepares outside any slot)."""
        from .lower import lds_layout

        if self.mode == D.M_DENSE_LDS:
            _, _, _, total = lds_layout(self.prog, 0 if self.shared else self.lds, UNROLL, BLOCK // 64)
            if total > 160 * 1024:
                self.mode, self.lds, self.hll_lds = D.M_DENSE_GLOBAL, 0, 0

    def _rows(self, cap: int) -> int:
        if self.mode == D.M_PART and self.part is not None and self.part.get("hashed"):
            return 1  # (sparse output: no group table)
        return cap if self.mode == D.M_HASH else self.prog.G

    def _geom(self, cap: int) -> tuple:
        """What a slot's device tensors look like (shapes and dtypes): prepared scans with equal
        geometry can hand each other their buffers."""
        prog = self.prog
        nblocks = prog.nhll_total if self.stored_fused else prog.nhll
        return (str(self.dev), self.mode, self._rows(cap), prog.nslots, nblocks, self.m, bool(self.hll32),
                bool(self.touch), bool(self.pres_bytes))

    def _alloc(self, cap: int, reuse: Optional["_Bufs"] = None) -> "_Bufs":
        """This slot's buffers -- the large tensors given by ``reuse`` (views of the slot's arena,
        whose contents are unknown: the first run resets them) or allocated here -- with this scan's
        own descriptor and launch arguments."""
        from .lower import lds_layout

        prog, dev = self.prog, self.dev
        b = _Bufs()
        b.cap = cap
        rows = self._rows(cap)
        b.rows = rows
        b.geom = self._geom(cap)
        b.init_row = _init_row(dev, tuple(int(init) for _, init in prog.slots))
        b.arena = None
        if reuse is not None and getattr(reuse, "geom", None) == b.geom:
            b.acc, b.keys, b.hll, b.hll32 = reuse.acc, reuse.keys, reuse.hll, reuse.hll32
            b.overflow, b.touch = reuse.overflow, reuse.touch
            if self.touch:
                b.touch.zero_()  # (the first-touch invariant: every byte clear between runs)
        else:
            b.hll, b.hll32 = [], []
            for name, n, dt, shape in self._tensor_layout(cap):
                t = torch.empty(n, dtype=dt, device=dev)
                t = t.view(shape) if shape is not None else t
                if name in ("hll", "hll32"):
                    getattr(b, name).append(t)
                else:
                    setattr(b, name, t)
            b.overflow = torch.zeros(1, dtype=torch.int32, device=dev)
            b.touch.zero_()
        b.clean = False
        hll_offs = []
        off = prog.G * prog.nslots * 8 * (BLOCK // 64)
        for _ in range(prog.nhll):
            hll_offs.append(off)
            off += prog.G * self.m * 4
        # (the shared-table layout lives in the JIT kernel only; the descriptor's interpreter layout
        # then carries no LDS accumulators)
        cache_off, wave_bytes, _, total = lds_layout(prog, 0 if self.shared else self.lds, UNROLL, BLOCK // 64)
        if total > 160 * 1024 and self.mode == D.M_DENSE_LDS:
            # accumulators + staging planes exceed the CU's LDS: accumulate in HBM instead
            self.mode, self.lds, self.hll_lds = D.M_DENSE_GLOBAL, 0, 0
            cache_off, wave_bytes, _, total = lds_layout(prog, 0, UNROLL, BLOCK // 64)
        if total > 160 * 1024:
            raise RuntimeError(f"query needs {total} bytes of LDS staging")
        d = pack(prog, self.mode, self.dedup, self.hll_lds, 0 if self.shared else self.lds, b.acc.data_ptr(),
                 b.keys.data_ptr(),
                 cap, b.overflow.data_ptr(), b.touch.data_ptr() if self.touch else 0, 0,
                 [h.data_ptr() for h in (b.hll32 or b.hll)], hll_offs,
                 unroll=UNROLL, cache_off=cache_off, wave_bytes=wave_bytes)
        self.lds_total = total
        self._total_chunks = int(d[0]["total_chunks"])
        self.grid = _grid(dev, self._total_chunks, self.jit.lay.total if self.jit else total, self.jit)
        b.part = None
        if self.mode == D.M_PART:
            b.part = self._part_bufs(d)
        b.desc = _upload(d.view(np.uint8), dev)
        b.run_args = b.noreset_args = None
        if self.mode not in (D.M_HASH, D.M_PART):
            # the whole launch path of one execution as cached arguments of ONE native call
            # (ops/csrc/bindings.cpp run_scan): fused reset of this slot's buffers + the kernel
            zeros = list(b.hll32 or b.hll) + ([b.touch] if self.touch else []) + ([b.acc] if self.pres_bytes else [])
            if len(zeros) <= 4 and all(z.numel() * z.element_size() % 8 == 0 for z in zeros):
                acc = None if self.pres_bytes else b.acc
                h = self.jit.handle if self.jit is not None else -1
                tail = (h, b.desc.data_ptr(), int(self.grid), BLOCK,
                        int(self.jit.lay.total if self.jit is not None else self.lds_total), UNROLL)
                b.run_args = (acc.data_ptr() if acc is not None else 0, b.init_row.data_ptr(),
                              int(acc.shape[0]) if acc is not None else 0, int(b.init_row.numel()),
                              [z.data_ptr() for z in zeros], [z.numel() * z.element_size() // 8 for z in zeros],
                              b.overflow.data_ptr()) + tail
                b.noreset_args = (0, 0, 0, 0, [], [], 0) + tail
        return b

    def _part_bufs(self, d) -> dict:
        """Record / count / offset buffers of the partitioned group-by for this slot; fills the
        descriptor's part_* fields (the producer's record regions and per-chunk end offsets)."""
        L, prog, dev = self.part, self.prog, self.dev
        u32 = torch.int32
        nch = int(d[0]["total_chunks"])
        cap = nch * D.CHUNK_ROWS            # chunk c owns records [4096 c, 4096 c + 4096)
        if cap * L["rw"] >= (1 << 32) or cap >= (1 << 32):
            raise RuntimeError("partitioned group-by: shard too large for u32 record offsets")
        P1, nsub = L["p1"], L["nsub"]
        # the producer counts its level-1 buckets itself (ops/jit.py part_hist_add): one histogram
        # column per producer block, and chunk end offsets stored in producer-block order
        # (jit.part_positions, empty padding positions stay 0), so the level-1 split's block k
        # scatters exactly producer block k's records -- no count pass over the records
        from ..ops import jit as J

        k1 = int(self.grid)
        npos, pos = J.part_positions(nch, k1)
        seg_lo = np.zeros(max(1, npos), dtype=np.int64)
        seg_lo[pos] = np.arange(nch, dtype=np.int64) * D.CHUNK_ROWS
        pb = {
            # the layout and producer grid these buffers and the descriptor were built for: a run
            # uses THEM, never the scan's current ones -- another slot running the same prepared
            # scan may re-layout it (hash overflow, observed group count) or swap in a specialized
            # kernel with another grid while this run is in flight, and mixing a new bucket count
            # with these buffers would write past them
            "L": L, "grid": int(self.grid),
            "cap_words": max(1, cap * L["rw"]), "desc_recs": 0,
            "seg_lo": torch.from_numpy(seg_lo).to(u32).to(dev),
            "pend": torch.zeros(max(1, npos), dtype=u32, device=dev),
            "k1": k1, "nch": nch, "npos": npos,
            "counts1": torch.empty(P1 * k1, dtype=u32, device=dev),
            "totals1": torch.empty(P1, dtype=u32, device=dev),
            "base1": torch.empty(P1 + 1, dtype=u32, device=dev),
        }
        if L["levels"] == 2:
            pb["counts2"] = torch.empty(nsub * L["k"], dtype=u32, device=dev)
            pb["totals2"] = torch.empty(nsub, dtype=u32, device=dev)
            pb["base2"] = torch.empty(nsub + 1, dtype=u32, device=dev)
        d[0]["part_recs"] = 0  # the slot's scratch, patched in at run time (_run_part)
        d[0]["part_counts"] = pb["pend"].data_ptr()
        d[0]["part_base"] = pb["counts1"].data_ptr()  # (the producer's histogram: [P1][grid])
        d[0]["part_shift"] = L["shift1"]
        d[0]["part_n"] = P1
        return pb

    def _run_part(self, b: "_Bufs") -> Optional[Partials]:
        """producer (records into chunk regions) -> level-1 split (count, offsets, tile-sorted
        scatter) -> [level-2 split] -> LDS aggregation into the dense table (every row written: no
        reset), or, with a fused HAVING, straight to the surviving groups (sparse)."""
        slab = PART_POOL.acquire(self.dev, b.part["cap_words"])
        try:
            return self._run_part_on(b, slab)
        finally:
            PART_POOL.release(slab)

    def _run_part_on(self, b: "_Bufs", slab: "_Slab") -> Optional[Partials]:
        nat, st = native.load(), native._stream(self.dev)
        pb = dict(b.part)
        L = pb["L"]
        prog = self.prog
        pb["recs1"], pb["recs2"] = slab.recs1, slab.recs2
        if b.part["desc_recs"] != pb["recs1"].data_ptr():
            off = D.SCANDESC.fields["part_recs"][1]
            ptr = torch.tensor([pb["recs1"].data_ptr()], dtype=torch.int64).view(torch.uint8)
            b.desc[off:off + 8].copy_(ptr.to(self.dev))
            b.part["desc_recs"] = pb["recs1"].data_ptr()
        # (the grid the histogram columns and chunk positions were laid out for: a kernel swapped in
        # since, with another resident grid, is still correct at this one -- it loops over chunks)
        jit = self.jit
        nat.module_launch(jit.handle, b.desc.data_ptr(), pb["grid"], BLOCK, int(jit.lay.total), st)
        rw, P1, k1 = L["rw"], L["p1"], pb["k1"]
        # level 1: one input group = every chunk region in producer-block order, block k of the
        # split = producer block k's chunks (their level-1 histogram came with the records)
        a1 = (pb["recs1"].data_ptr(), rw, pb["seg_lo"].data_ptr(), pb["pend"].data_ptr(), 1, pb["npos"], k1,
              L["shift1"], P1, pb["counts1"].data_ptr())
        # dense keys arrive in runs (rows in time order, then key order within a day): the split
        # kernels' same-bucket waves add once (partition.hip lds_count_add); hashes are uniform
        cl = 0 if L.get("hashed") else 2
        nat.part_scan(pb["counts1"].data_ptr(), P1, k1, pb["totals1"].data_ptr(), pb["base1"].data_ptr(), st)
        # (a small value field packed into the key word above shift1: one word less per record for
        # every later pass -- part_layout "pack")
        pk = L.get("pack")
        nat.part_split(*a1, pb["base1"].data_ptr(), pb["recs2"].data_ptr(), 1 | cl | ((pk[1] if pk else 0) << 8), st)
        rw = L.get("rw1", rw)
        fields = L.get("agg_fields", L["fields"])
        recs, base = pb["recs2"], pb["base1"]
        if L["levels"] == 2:
            # level 2: group p = level-1 bucket p (one segment [base1[p], base1[p+1])), P2 sub-buckets
            b1 = pb["base1"].data_ptr()
            a2 = (pb["recs2"].data_ptr(), rw, b1, b1 + 4, P1, 1, L["k"], L["shift"], L["p2"],
                  pb["counts2"].data_ptr())
            nat.part_split(*a2, 0, 0, cl, st)
            nat.part_scan(pb["counts2"].data_ptr(), L["nsub"], L["k"], pb["totals2"].data_ptr(),
                          pb["base2"].data_ptr(), st)
            nat.part_split(*a2, pb["base2"].data_ptr(), pb["recs1"].data_ptr(), 1 | cl, st)
            recs, base = pb["recs1"], pb["base2"]
        if L.get("hashed"):
            return self._run_part_hashed(b, recs, base)
        hv, tk = self.part_having, self.part_topk
        if hv is None and tk is None:
            # (HLL aggregators: each sub-bucket also writes its groups' rows of the register tables)
            nat.part_agg_hll(recs.data_ptr(), rw, base.data_ptr(), L["nsub"], int(prog.G), L["shift"],
                             [f[0] for f in fields], [f[1] for f in fields],
                             [int(op) for op, _ in prog.slots], [int(init) for _, init in prog.slots],
                             b.acc.data_ptr(), [], 1, 0, 0, 0, [h.data_ptr() for h in b.hll] if L.get("nhll") else [],
                             int(prog.hll_p), st, self._stored_csr() if L.get("nhll") else [])
            return None
        terms, conj = hv if hv is not None else ([], 1)
        while True:
            acc, keys, cnt, _ = self._sparse_out(b, "hv_out", False)
            args = (recs.data_ptr(), rw, base.data_ptr(), L["nsub"], int(prog.G), L["shift"],
                    [f[0] for f in fields], [f[1] for f in fields], [int(op) for op, _ in prog.slots],
                    [int(init) for _, init in prog.slots], acc.data_ptr(), terms, conj, keys.data_ptr(),
                    cnt.data_ptr(), int(acc.shape[0]))
            if tk is not None:
                # ORDER BY <aggregate> LIMIT k in the same kernel: a few candidates per sub-bucket
                # (every tie kept) instead of every surviving group, no radix select after it
                nat.part_agg_topk(*args, *tk, st)
            else:
                nat.part_agg(*args, st)
            # (the whole partition pipeline: one copy + one sleeping wait, not a spin + a round trip)
            n = int(native.read_words([cnt], self.dev)[0])
            if n <= acc.shape[0]:
                return Partials("sparse", acc[:n], keys[:n], [])
            self.part_cap = _next_pow2(n + n // 4)  # more survivors than room: grow, aggregate again

    def _stored_csr(self) -> list:
        """(offsets, pairs) device pointers of each stored sketch metric, in register-table order."""
        ds = self.prog.ds
        out = []
        for _, metric, _ in self.prog.stored_hll:
            sk = ds.metrics[metric].sketch
            if sk.offsets.device != self.dev or sk.values.device != self.dev or sk.offsets.dtype != torch.int64 \
                    or sk.values.dtype != torch.int32:
                raise RuntimeError(f"stored sketch {metric!r} is not a device int64/int32 CSR")
            out.append((sk.offsets.data_ptr(), sk.values.data_ptr()))
        return out

    def _run_part_hashed(self, b: "_Bufs", recs: torch.Tensor, base: torch.Tensor) -> Partials:
        """Sparse LDS-hash aggregation of the hash-partitioned records (keys beyond 32 bits).  A
        sub-bucket that held more distinct keys than its table (the planner's group estimate was
        low) makes the whole execution re-partition into 4x more sub-buckets and run again."""
        L, nat, st, prog = b.part["L"], native.load(), native._stream(self.dev), self.prog
        hv = self.part_having or ([], 1)
        while True:
            acc, keys, cnt, ovf, hll = self._sparse_out(b, "hh_out", True, L.get("nhll", 0))
            nat.part_hash_agg_hll(recs.data_ptr(), L["rw"], base.data_ptr(), L["nsub"], L["cap_log2"],
                                  [f[0] for f in L["fields"]], [f[1] for f in L["fields"]],
                                  [int(op) for op, _ in prog.slots], [int(init) for _, init in prog.slots], hv[0],
                                  hv[1], keys.data_ptr(), acc.data_ptr(), cnt.data_ptr(), int(acc.shape[0]),
                                  ovf.data_ptr(), [h.data_ptr() for h in hll], int(prog.hll_p), st)
            n, overflow = (int(x) for x in native.read_words([cnt, ovf], self.dev))
            if overflow:
                if L["scale"] >= 1 << 12:
                    raise RuntimeError("hash-partitioned group-by: sub-bucket overflow persists")
                with self._slot_lock:
                    self.part = L = part_hash_layout(prog, L["scale"] * 4)
                    self._slots.clear()
                nb = self._bufs()
                return self._run_part(nb) if nb.part is not None else self._empty()
            if n <= acc.shape[0]:
                if not hv[0] and n * 8 < L["nsub"] << (L["cap_log2"] - 1):
                    # far fewer groups than the row estimate sized for (TPC-H Q16: 12M groups of
                    # 554M estimated rows -> 262k sub-buckets, each LDS table 128 KB for ~45 keys,
                    # 8.5 ms of table init and emit): later runs partition for the observed count
                    with self._slot_lock:
                        self.part = part_hash_layout(prog, L["scale"], groups=1.25 * n)
                        self._slots.clear()
                return Partials("sparse", acc[:n], keys[:n], [h[:n] for h in hll])
            self.part_cap = _next_pow2(n + n // 4)  # more groups than room: grow, aggregate again

    def _sparse_out(self, b: "_Bufs", name: str, ovf: bool, nhll: int = 0) -> tuple:
        """(acc [part_cap][nslots], keys, count[, overflow], [hll [part_cap][2^p] x nhll]) the
        partitioned aggregation appends its surviving groups to: carved from the slot's arena on a
        leased slot (they live as long as the statement's partials), cached on the buffers on slot 0.
        (Counts are reset by the launch.)"""
        cap, ns, dev, m = self.part_cap, self.prog.nslots, self.dev, self.m
        slot = current_slot()
        if slot == 0:
            out = b.part.get(name)
            if out is None or out[0].shape[0] < cap or len(out[-1]) != nhll:
                out = b.part[name] = (torch.empty((cap, ns), dtype=torch.int64, device=dev),
                                      torch.empty(cap, dtype=torch.int64, device=dev),
                                      torch.zeros(2, dtype=torch.int64, device=dev)) + \
                    ((torch.zeros(1, dtype=torch.int32, device=dev),) if ovf else ()) + \
                    ([torch.empty((cap, m), dtype=torch.uint8, device=dev) for _ in range(nhll)],)
            return out
        # (the count word is followed by a fused top-k's threshold word)
        items = [(cap * ns, torch.int64, (cap, ns)), (cap, torch.int64, None), (2, torch.int64, None)] + \
            ([(1, torch.int32, None)] if ovf else []) + [(cap * m, torch.uint8, (cap, m))] * nhll
        offs, total = _carve_aligned([n * torch.empty((), dtype=dt).element_size() for n, dt, _ in items])
        _, off, _, buf = slot_arena(dev, slot).carve(total, self)
        views = [SlotArena.view(buf, off + o, n, dt, shape) for (n, dt, shape), o in zip(items, offs)]
        k = 4 if ovf else 3
        return tuple(views[:k]) + (views[k:],)

    def set_part_topk(self, k: int, slot: int, is_f64: bool, desc: bool) -> bool:
        """Fuse a groupBy ORDER BY <aggregate slot> LIMIT k into the partitioned aggregation
        (engine/executor.py _fuse_topk): each sub-bucket emits only groups at or above its k-th best
        and the best k-th an earlier sub-bucket published -- a superset of the top k with every
        tie, ordered and limited exactly afterwards.  False when this scan cannot (hash-keyed and
        sketch layouts keep the radix select after the aggregation)."""
        L = self.part or {}
        if self.mode != D.M_PART or not (1 <= int(k) <= 16) or L.get("nhll") or L.get("hashed") or \
                not (0 <= int(slot) < self.prog.nslots) or L.get("shift", 99) > 12:
            return False  # (the kernel ranks tables of at most 4096 keys: 8 rows per thread)
        self.part_topk = (int(k), int(slot), 1 if is_f64 else 0, 1 if desc else 0)
        return True

    def set_part_having(self, terms, conj: bool) -> bool:
        """Fuse a groupBy HAVING into the partitioned aggregation (engine/executor.py): only existing
        groups passing it leave the kernel, as sparse partials.  terms: [(slot, is_f64, op, divisor,
        constant)], op 0 equalTo / 1 greaterThan / 2 lessThan.  False when this scan cannot."""
        if self.mode != D.M_PART or not terms or len(terms) > 4 or (self.part or {}).get("nhll"):
            return False
        self.part_having = ([tuple(t) for t in terms], 1 if conj else 0)
        return True

    def _launch(self, b: "_Bufs"):
        if self.jit is not None:
            self.jit.launch(b.desc, self.grid)
        else:
            native.scan(b.desc, self.grid, BLOCK, self.lds_total, UNROLL)

    def _reset(self, b: "_Bufs"):
        if self.touch and b.clean:
            return  # the previous run re-initialised exactly the rows it touched
        # one fused launch (ops/csrc/post_scan.hip reset_bufs_kernel) instead of a fill per buffer
        zeros = list(b.hll32 or b.hll)
        if self.touch:
            zeros.append(b.touch)
        acc = b.acc
        if self.pres_bytes:
            zeros.append(b.acc)
            acc = None
        if len(zeros) <= 4:
            native.reset_bufs(acc, b.init_row, zeros, b.overflow)
        else:
            if acc is not None:
                acc.copy_(b.init_row.expand_as(acc))
            for z in zeros:
                z.zero_()
            b.overflow.zero_()
        if self.mode == D.M_HASH:
            b.keys.fill_(-1)

    # ------------------------------------------------------------------ specialization
    def _maybe_specialize(self) -> None:
        self._runs += 1
        fut = self._spec_future
        if fut is not None and fut.done():
            self._spec_future = None
            try:
                self._adopt(fut.result())
            except Exception as e:  # noqa: BLE001  (keep the shared kernel)
                import warnings

                warnings.warn(f"literal specialization failed: {e}")
        if self._runs < self._spec_at or SPECIALIZE == "off" or self.jit is None or self.jit.literals:
            return
        if SPECIALIZE == "sync":
            self._spec_at = 1 << 62
            self._adopt(self.jit.specialized())
            return
        with _spec_lock:
            if _spec_pending[0] >= SPEC_MAX_PENDING:
                self._spec_at = 2 * self._runs  # the compile queue is full: ask again later
                return
            _spec_pending[0] += 1
        self._spec_at = 1 << 62
        self._spec_future = _spec_executor().submit(_spec_job, self.jit)
        from ..utils.metrics import count_event

        count_event("jit_spec_submit")

    def _adopt(self, js) -> None:
        """Swap in a kernel of the same layout (the launch arguments cached per slot name the
        kernel handle)."""
        with self._slot_lock:
            self.jit = js
            if getattr(self, "_total_chunks", None) is not None:
                # the specialized kernel's register use may allow a different resident grid
                self.grid = _grid(self.dev, self._total_chunks, js.lay.total, js)
            for b in self._slots.values():
                for attr in ("run_args", "noreset_args"):
                    a = getattr(b, attr)
                    if a is not None:
                        a = list(a)
                        a[-6] = js.handle  # (jit, desc, grid, block, lds, unroll)
                        a[-4] = int(self.grid)
                        setattr(b, attr, tuple(a))
        from ..utils.metrics import count_event

        count_event("jit_spec_adopt")

    # ------------------------------------------------------------------ run
    def run(self) -> Partials:
        self._maybe_specialize()
        prog = self.prog
        b = self._bufs()
        if prog.empty:
            if self.mode != D.M_HASH:
                # dense layout even when this shard has nothing to scan: every rank must issue the
                # same merge collective (parallel/merge.py) for the same query
                self._reset(b)
                for h in (b.hll if b.hll32 else []):
                    h.zero_()
                return Partials("dense", b.acc, None, [h.view(b.rows, self.m) for h in b.hll])
            return self._empty()
        while True:
            if b.run_args is not None:
                native.run_scan(*(b.noreset_args if (self.touch and b.clean) else b.run_args),
                                native._stream(self.dev))
            elif self.mode == D.M_PART:
                sp = self._run_part(b)
                if sp is not None:
                    return sp
            else:
                self._reset(b)
                self._launch(b)
            b.clean = False  # dirty until the touched rows are re-initialised below
            for h8, h32 in zip(b.hll, b.hll32):  # scan-time u32 registers -> the byte registers
                h8.copy_(h32)
            if self.touch:
                # touched groups' ids and rows, re-initialised in the same pass (post_scan.hip touch_*)
                idx, acc = native.touch_compact(b.touch, b.acc, b.init_row)
                b.clean = True
                return Partials("sparse", acc, idx, [])
            if self.pres_bytes:
                idx = native.nonzero_rows(b.acc)
                return Partials("sparse", torch.ones((idx.numel(), 1), dtype=torch.int64, device=self.dev), idx, [])
            if self.mode != D.M_HASH:
                break
            if int(b.overflow.item()) == 0:
                break
            b = self._rebuf(b.cap * 4)  # grow and retry
            self.cap = max(self.cap, b.cap)
        if self.mode == D.M_HASH:
            valid = _nonzero_big(b.keys != -1)
            out = Partials("sparse", b.acc.index_select(0, valid), b.keys.index_select(0, valid),
                           [h.view(b.rows, self.m).index_select(0, valid) for h in b.hll])
            # adaptive capacity: the planner's row estimate sizes the first table (TPC-H Q16's NOT
            # filters: 2^31 slots for 12M groups); later runs of this prepared query size it from
            # the observed group count (an overflow still grows it and retries)
            want = _next_pow2(2 * int(valid.numel()) + 1024)
            if want * 4 <= b.cap:
                self.cap = want
                self._rebuf(want)
            return out
        return Partials("dense", b.acc, None, [h.view(b.rows, self.m) for h in b.hll])

    def fast_launch(self) -> Optional["_Bufs"]:
        """``run()`` of a dense-LDS scan with a fused launch (engine/executor.py _SmallDenseRunner):
        the slot's buffers after the reset + kernel are enqueued, or None when this slot's buffers
        have no fused launch (the caller then takes ``run()``)."""
        self._maybe_specialize()
        b = self._bufs()
        if b.run_args is None or b.hll32:
            return None
        # clean: the previous fast run re-initialised the buffers behind its result copy
        native.run_scan(*(b.noreset_args if b.clean else b.run_args), native._stream(self.dev))
        b.clean = False
        return b

    # single-slot views (tests and tools inspect the implicit slot's buffers)
    @property
    def acc(self):
        return self._bufs().acc

    @property
    def desc(self):
        return self._bufs().desc

    def _empty(self) -> Partials:
        prog = self.prog
        acc = torch.empty((0, prog.nslots), dtype=torch.int64, device=self.dev)
        return Partials("sparse", acc, torch.zeros(0, dtype=torch.int64, device=self.dev),
                        [torch.zeros((0, self.m), dtype=torch.uint8, device=self.dev)
                         for _ in range(prog.nhll_total if self.stored_fused else prog.nhll)])


# ------------------------------------------------------------------------------------------------
# Device-buffer budget across prepared scans.  Plans stay cached (a dashboard's thousands of
# parameterizations), but their per-slot device buffers -- a 150M-group table is 1.2-2.4 GB -- are
# released least-recently-used first once all prepared scans together hold more than the budget;
# a released scan re-allocates on its next run (from the caching allocator's free blocks, usually:
# parameterizations of one shape have the same buffer sizes).  Callers still holding partials keep
# those tensors alive by reference, so a release never pulls memory from under a running query.
BUF_BUDGET = int(os.environ.get("SDO_SCAN_BUF_BUDGET", "0"))  # 0: 35% of the device's memory


HEADROOM = 16 << 30  # device memory kept free for a statement's temporaries (sorts, gathers, results)


def _budget() -> int:
    """Bytes the cached per-slot scan buffers may hold: 35% of the device, and never more than what
    is left once everything else allocated (the resident shards, the partition scratch of every
    slot, results in flight) and ``HEADROOM`` are accounted for -- a many-client BI workload over
    hundreds of statements with 150M-group tables otherwise grows into an out-of-memory error."""
    if BUF_BUDGET > 0:
        return BUF_BUDGET
    b = _budget_cache.get("b")
    total = _budget_cache.get("total")
    if b is None:
        b, total = 24 << 30, 0
        try:
            if torch.cuda.is_available():
                total = int(torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory)
                b = max(b, int(0.35 * total))
        except Exception:  # noqa: BLE001
            pass
        _budget_cache["b"], _budget_cache["total"] = b, total
    if total:
        other = torch.cuda.memory_allocated() - _buf_total[0]
        b = min(b, max(1 << 30, total - other - HEADROOM))
    return b


_budget_cache: dict = {}

# Partition records (ops/csrc/partition.hip) are scratch of one execution: two record buffers
# (producer regions / split output), sized for every row of the scanned chunks -- 4.8-14 GB at SF100.
# Held per execution slot they multiplied by the slot count (6 slots of a BI plan: ~86 GB); instead
# one device-wide pool hands out slabs under a byte budget.  A slab goes back to the pool once the
# execution's kernels are enqueued, with an event on its stream: the next holder's stream waits for
# that event, so the memory is reused in device order without a host sync.  A thread already
# holding a slab never waits for another (a hashed re-partition takes a second one over budget).
PART_SCRATCH_BUDGET = int(os.environ.get("SDO_PART_SCRATCH_BUDGET", "0"))  # 0: 12% of the device


class _Slab:
    __slots__ = ("dev", "recs1", "recs2", "words", "event")


class PartScratchPool:
    def __init__(self):
        self.cv = threading.Condition()
        self.free: List[_Slab] = []
        self.total = 0
        self.held = threading.local()
        self.peak_words: dict = {}  # device -> largest slab asked for (presize)

    def _budget(self, dev) -> int:
        if PART_SCRATCH_BUDGET > 0:
            return PART_SCRATCH_BUDGET
        try:
            return int(0.12 * torch.cuda.get_device_properties(dev).total_memory)
        except Exception:  # noqa: BLE001
            return 32 << 30

    def acquire(self, dev, words: int) -> _Slab:
        """Two u32 record buffers of at least ``words`` each; the current stream waits for the
        slab's previous holder."""
        words = max(1, int(words))
        need = 2 * words * 4
        depth = getattr(self.held, "n", 0)
        with self.cv:
            if words > self.peak_words.get(str(dev), 0):
                self.peak_words[str(dev)] = words
            while True:
                fit = [x for x in self.free if x.dev == str(dev) and x.words >= words]
                if fit:
                    sl = min(fit, key=lambda x: x.words)
                    self.free.remove(sl)
                    break
                # drop free slabs too small (or of another device) while the new one does not fit
                while self.free and self.total + need > self._budget(dev):
                    x = self.free.pop(0)
                    self.total -= 2 * x.words * 4
                if self.total + need <= self._budget(dev) or self.total == 0 or depth > 0:
                    sl = None
                    self.total += need
                    break
                self.cv.wait(timeout=1.0)
        if sl is None:
            try:
                sl = _Slab()
                sl.dev, sl.words, sl.event = str(dev), words, None
                sl.recs1 = _with_eviction(lambda: shared_empty(words, torch.int32, dev), None, None)
                sl.recs2 = _with_eviction(lambda: shared_empty(words, torch.int32, dev), None, None)
                from ..utils.metrics import count_event

                count_event("part_slab_alloc")
            except BaseException:
                with self.cv:
                    self.total -= need
                    self.cv.notify_all()
                raise
        if sl.recs1.is_cuda:
            cs = torch.cuda.current_stream(sl.recs1.device)
            if sl.event is not None:
                cs.wait_event(sl.event)
            # slabs move between slot streams: the caching allocator must not hand their blocks to
            # an allocation of the stream they were made on while this stream's kernels still use
            # them (a slab dropped from the pool is freed at once)
            sl.recs1.record_stream(cs)
            sl.recs2.record_stream(cs)
        self.held.n = depth + 1
        return sl

    def release(self, sl: _Slab) -> None:
        if sl.recs1.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(sl.recs1.device))
            sl.event = ev
        self.held.n = max(0, getattr(self.held, "n", 1) - 1)
        with self.cv:
            self.free.append(sl)
            self.cv.notify_all()

    def presize(self, dev, nslots: int) -> int:
        """Free slabs of the largest size acquired so far until ``nslots`` of them exist (or the
        budget is spent); returns how many were added.  (Warm-up only: no slab is held.)"""
        from ..utils.metrics import count_event

        words = self.peak_words.get(str(dev), 0)
        if words <= 0:
            return 0
        added = 0
        with self.cv:
            keep = []
            for x in self.free:
                if x.dev == str(dev) and x.words < words:
                    self.total -= 2 * x.words * 4  # too small for the largest run: replaced below
                else:
                    keep.append(x)
            self.free = keep
            have = sum(1 for x in self.free if x.dev == str(dev))
            while have < nslots and self.total + 2 * words * 4 <= self._budget(dev):
                sl = _Slab()
                sl.dev, sl.words, sl.event = str(dev), words, None
                sl.recs1 = shared_empty(words, torch.int32, dev)
                sl.recs2 = shared_empty(words, torch.int32, dev)
                self.total += 2 * words * 4
                self.free.append(sl)
                have += 1
                added += 1
                count_event("part_slab_presize")
            self.cv.notify_all()
        return added

    def clear(self) -> None:
        with self.cv:
            for x in self.free:
                self.total -= 2 * x.words * 4
            self.free = []
            self.cv.notify_all()

    def bytes(self) -> int:
        return self.total


PART_POOL = PartScratchPool()


_buf_lru: "OrderedDict[tuple, tuple]" = OrderedDict()   # (id(prep), slot) -> (weakref(prep), bytes)
_buf_total = [0]
_buf_lock = threading.Lock()


def _bufs_nbytes(b: "_Bufs") -> int:
    n = 0
    for t in [b.acc, b.keys, b.overflow, b.desc, b.touch, b.init_row] + list(b.hll) + list(b.hll32 or []):
        n += t.numel() * t.element_size()
    for v in (b.part or {}).values():
        if isinstance(v, torch.Tensor):
            n += v.numel() * v.element_size()
        elif isinstance(v, tuple):
            n += sum(t.numel() * t.element_size() for t in v if isinstance(t, torch.Tensor))
    return n


def _buffers_acquired(prep, slot, b) -> None:
    key = (id(prep), slot)
    nb = _bufs_nbytes(b)
    victims = []
    budget = _budget()  # (outside the lock: it allocates)
    with _buf_lock:
        _settle_forgotten()
        old = _buf_lru.pop(key, None)
        if old is not None:
            _buf_total[0] -= old[1]
        _buf_lru[key] = (weakref.ref(prep), nb)
        _buf_total[0] += nb
        while _buf_total[0] > budget and len(_buf_lru) > 1:
            k, (ref, n) = next(iter(_buf_lru.items()))
            if k == key:
                break
            _buf_lru.pop(k)
            _buf_total[0] -= n
            victims.append((ref(), k[1]))
    for p, sl in victims:
        if p is not None:
            with p._slot_lock:
                p._slots.pop(sl, None)


def release_device_memory(keep=None, keep_arena=None) -> None:
    """Drop every prepared scan's cached slot buffers (but ``keep``'s (prep, slot)), the other slots'
    arenas (but ``keep_arena``), the shared scratch and the allocator's free blocks.  A scan running
    on a dropped slot keeps its tensors alive through its own references until it finishes."""
    from ..utils.metrics import count_event

    count_event("device_memory_release")
    for ar in list(_ARENAS.values()):
        if ar is not keep_arena and ar.slot != (keep[1] if keep else None):
            ar.release(blocking=False)
    victims = []
    with _buf_lock:
        for k in list(_buf_lru):
            if k == keep:
                continue
            ref, n = _buf_lru.pop(k)
            _buf_total[0] -= n
            victims.append((ref(), k[1]))
    for p, sl in victims:
        if p is not None:
            with p._slot_lock:
                p._slots.pop(sl, None)
    PART_POOL.clear()
    torch.cuda.empty_cache()


def _with_eviction(fn, prep, slot, arena=None):
    """Run an allocation; on a device out-of-memory error release every other prepared scan's
    cached slot buffers, the other slots' arenas and the allocator's free blocks, then try once
    more."""
    try:
        return fn()
    except torch.OutOfMemoryError:
        import logging

        logging.getLogger(__name__).warning("device out of memory on slot %s: releasing cached buffers", slot)
        release_device_memory(keep=(id(prep), slot), keep_arena=arena)
        return fn()


def _buffers_used(prep, slot) -> None:
    key = (id(prep), slot)
    with _buf_lock:
        if key in _buf_lru:
            _buf_lru.move_to_end(key)


_forgotten: list = []  # ids of collected prepared scans, settled under _buf_lock by the next user


def _forget_prep(pid: int) -> None:
    """A prepared scan was collected: its buffers went with it.  (A finalizer: it may run inside
    any allocation -- including one made while this thread holds ``_buf_lock`` -- so it only
    records the id; ``_settle_forgotten`` drops the accounting under the lock.)"""
    _forgotten.append(pid)


def _settle_forgotten() -> None:
    """(caller holds _buf_lock)"""
    while _forgotten:
        pid = _forgotten.pop()
        for k in [k for k in _buf_lru if k[0] == pid]:
            _buf_total[0] -= _buf_lru.pop(k)[1]


class _Bufs:
    """One execution slot's device buffers for a prepared scan."""
    __slots__ = ("cap", "rows", "init_row", "acc", "keys", "hll", "hll32", "overflow", "desc", "touch", "clean",
                 "run_args", "noreset_args", "part", "geom", "arena", "__weakref__")


# Slot arenas.  A BI dashboard sends many statement shapes and parameterizations; caching one set of
# device tables per (prepared scan, slot) made the slots' memory the SUM over every plan ever run
# (the reference's JMeter BI plan at 6 slots: 262 GiB allocated, out of memory).  A leased slot runs
# one statement at a time (engine/scheduler.py), so its scans carve their large tensors from one
# per-slot arena instead: a bump allocation that restarts with every statement on the slot
# (``slot_epoch``), grown to the slot's largest statement -- K slots hold K x the largest need.
# A scan keeps its descriptor while it lands at the same arena offset (a repeated statement carves
# in the same order: the same offsets every time); its first-touch / "reset behind the copy" state
# survives when nothing else was carved over its region since its last run, and is reset otherwise.
# Slot 0 (unleased callers: scripts, tests, the bench) keeps per-scan buffers under the LRU budget.
ARENA_ALIGN = 256
ARENA_MIN = 64 << 20

# Long-lived scratch (slot arena storages, partition slabs) is allocated on ONE allocation stream
# per device and marked used by each stream that runs on it (``record_stream``).  The caching
# allocator keeps a freed block for reuse by allocations of the stream it was made on only: made on
# the 8 slot streams, every arena growth step and dropped slab stayed cached on its own slot's
# stream, unusable by the others' next (larger) growth, until the allocator hit the device cap and
# freed everything with the device synchronised -- a 3.3 s freeze of every slot in the cold BI
# burst (profiles/r6/cold_burst_notes.md).  On one stream the dropped storages are the next
# growth's free blocks.
_ALLOC_STREAMS: dict = {}


def _alloc_stream(dev) -> "torch.cuda.Stream":
    k = str(dev)
    s = _ALLOC_STREAMS.get(k)
    if s is None:
        with _arena_lock:
            s = _ALLOC_STREAMS.get(k)
            if s is None:
                s = _ALLOC_STREAMS[k] = torch.cuda.Stream(torch.device(dev))
    return s


def shared_empty(n: int, dtype, dev) -> torch.Tensor:
    """``torch.empty`` of long-lived scratch on the device's allocation stream, recorded as used by
    the current stream (callers record any further stream that runs on it)."""
    dev = torch.device(dev)
    if dev.type != "cuda":
        return torch.empty(n, dtype=dtype, device=dev)
    cur = torch.cuda.current_stream(dev)
    with torch.cuda.stream(_alloc_stream(dev)):
        t = torch.empty(n, dtype=dtype, device=dev)
    t.record_stream(cur)
    return t


class SlotArena:
    """One execution slot's device memory for the scans of its current statement."""

    def __init__(self, dev, slot: int):
        self.dev, self.slot = dev, slot
        self.buf: Optional[torch.Tensor] = None   # uint8 storage
        self.cap = 0
        self.gen = 0          # storage generation (a new storage on growth / release)
        self.epoch = -1       # the slot's statement epoch the bump pointer belongs to
        self.off = 0
        self.need = 0         # bytes the current statement carved so far (across growths)
        self.binds: dict = {}  # start -> (end, owner id) of the regions' last carvers (current gen)
        self.users: "weakref.WeakSet" = weakref.WeakSet()  # scans holding views of this storage
        self.rec: set = set()  # streams the current storage is recorded as used by
        self.lock = threading.Lock()  # (release_device_memory may drop the storage from another thread)

    def carve(self, nbytes: int, owner) -> tuple:
        """(gen, offset, intact, storage) of ``nbytes`` for ``owner`` in the current statement:
        ``intact`` when the region was last carved by the same owner with the same size and nothing
        carved over it since (its contents are as that owner left them).  Views are taken from the
        returned storage (another thread's out-of-memory release may drop the arena's own reference
        at any time)."""
        with self.lock:
            r = self._carve(nbytes, owner)
            return r + (self.buf,)

    def _carve(self, nbytes: int, owner) -> tuple:
        from .scheduler import slot_epoch

        ep = slot_epoch(self.slot)
        if ep != self.epoch:
            self.epoch, self.off, self.need = ep, 0, 0
        nbytes = (max(1, nbytes) + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN
        self.need += nbytes
        if self.off + nbytes > self.cap:
            # the earlier scans of this statement keep the old storage alive through their views;
            # the next statement on the slot fits the new one whole.  Every slot runs every kind of
            # statement sooner or later: a growing arena goes straight to the largest peer's size
            # (one growth per slot, not a doubling series whose dropped steps stay in the caching
            # allocator's per-stream pools until a free-everything retry)
            peer = 0
            if _ARENAS.get((str(self.dev), self.slot)) is self:
                peer = max((a.cap for k, a in list(_ARENAS.items()) if k[0] == str(self.dev)), default=0)
            cap = max(ARENA_MIN, 2 * self.cap, self.need, peer)
            cap = (cap + ARENA_MIN - 1) // ARENA_MIN * ARENA_MIN
            self._drop()
            self.buf = _with_eviction(lambda: shared_empty(cap, torch.uint8, self.dev), None, self.slot, arena=self)
            self.cap = cap
            from ..utils.metrics import count_event

            count_event("arena_grow")
        if self.buf.is_cuda:  # (a storage presized on the warm-up thread's stream runs on the slot's)
            cs = torch.cuda.current_stream(self.buf.device)
            if cs.cuda_stream not in self.rec:
                self.buf.record_stream(cs)
                self.rec.add(cs.cuda_stream)
        start = self.off
        self.off += nbytes
        end = start + nbytes
        intact = self.binds.get(start) == (end, id(owner))
        for st in [st for st, (e, _) in self.binds.items() if st < end and e > start]:
            del self.binds[st]
        self.binds[start] = (end, id(owner))
        self.users.add(owner)
        return self.gen, start, intact

    @staticmethod
    def view(buf: torch.Tensor, off: int, nelem: int, dtype, shape=None) -> torch.Tensor:
        nb = nelem * torch.empty((), dtype=dtype).element_size()
        t = buf[off:off + nb].view(dtype)
        return t.view(shape) if shape is not None else t

    def release(self, blocking: bool = True) -> bool:
        """Drop the storage; ``blocking=False`` skips an arena whose lock is held (an out-of-memory
        release from another slot: that slot may itself be carving -- growing under its lock -- and
        waiting on this thread's arena in its own release, a lock-order deadlock)."""
        if not self.lock.acquire(blocking=blocking):
            return False
        try:
            self._drop()
        finally:
            self.lock.release()
        return True

    def _drop(self) -> None:
        """Forget the storage: scans holding views re-carve at their next run (running statements
        keep their tensors alive by reference until they finish)."""
        for p in list(self.users):
            with p._slot_lock:
                p._slots.pop(self.slot, None)
        self.users = weakref.WeakSet()
        self.buf, self.cap, self.off = None, 0, 0
        self.binds = {}
        self.rec = set()
        self.gen += 1


_ARENAS: dict = {}
_arena_lock = threading.Lock()


def slot_arena(dev, slot: int) -> SlotArena:
    k = (str(dev), slot)
    ar = _ARENAS.get(k)
    if ar is None:
        with _arena_lock:
            ar = _ARENAS.setdefault(k, SlotArena(dev, slot))
    return ar


def presize_device_memory(dev=None, nslots: int = 0) -> dict:
    """Server warm-up: grow every slot arena (1..``nslots``) to the largest one's size and fill the
    partition scratch pool to one slab per slot at its largest slab, then hand the caching
    allocator's free blocks -- the growth steps the warm-up statements left in per-stream pools --
    back to the device.  After this a warmed statement mix carves from storage that exists: no
    arena grows, no slab is allocated and the allocator never reaches the device cap and frees
    everything mid-service (a free-all retry synchronises the device under the allocator's lock
    while the allocating thread holds the GIL: every slot stalls for 1-2 s --
    profiles/r6/thrift_jmx_q250_stalls.md).  Call it with no statement running (the arenas'
    storages are replaced)."""
    from ..utils.metrics import count_event

    if not torch.cuda.is_available():
        return {}
    dev = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
    mine = [a for k, a in list(_ARENAS.items()) if k[0] == str(dev)]
    peak = max((a.cap for a in mine), default=0)
    grown = 0
    if peak > 0:
        for slot in range(1, max(0, int(nslots)) + 1):
            ar = slot_arena(dev, slot)
            with ar.lock:
                if ar.cap < peak:
                    ar._drop()
                    ar.buf = shared_empty(peak, torch.uint8, dev)
                    ar.cap = peak
                    grown += 1
                    count_event("arena_presize")
    slabs = PART_POOL.presize(dev, nslots)
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return {"arenas_grown": grown, "arena_gb": round(peak / 1e9, 3), "slabs_added": slabs,
            "reserved_gb": round(torch.cuda.memory_reserved(dev) / 1e9, 2),
            "allocated_gb": round(torch.cuda.memory_allocated(dev) / 1e9, 2)}


def arena_bytes() -> int:
    """Device bytes held by the slot arenas (their current storages)."""
    return sum(a.cap for a in list(_ARENAS.values()))


def device_memory_report() -> dict:
    """Where the device memory is (GB): the allocator's totals, the slot arenas, the partition
    scratch, the slot-0 cached scan buffers, and the release / retry events so far."""
    from ..utils.metrics import events

    g = 1e9
    out = {"arenas_gb": round(arena_bytes() / g, 3),
           "arena_per_slot_gb": {f"{k[1]}": round(a.cap / g, 3) for k, a in sorted(_ARENAS.items(), key=lambda x: x[0][1])},
           "part_scratch_gb": round(PART_POOL.bytes() / g, 3),
           "slot0_bufs_gb": round(_buf_total[0] / g, 3), "events": events()}
    if torch.cuda.is_available():
        ms = torch.cuda.memory_stats()
        out.update(allocated_gb=round(torch.cuda.memory_allocated() / g, 2),
                   reserved_gb=round(torch.cuda.memory_reserved() / g, 2),
                   max_allocated_gb=round(torch.cuda.max_memory_allocated() / g, 2),
                   # the caching allocator's free-everything-and-retry passes (each frees every cached
                   # block of every stream: a device-wide stall) and its device allocations / frees
                   alloc_retries=int(ms.get("num_alloc_retries", 0)), device_allocs=int(ms.get("num_device_alloc", 0)),
                   device_frees=int(ms.get("num_device_free", 0)))
    return out


def _carve_aligned(sizes: List[int]) -> tuple:
    offs, off = [], 0
    for n in sizes:
        offs.append(off)
        off += (max(1, n) + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN
    return offs, off


class PreparedEmit:
    """(group key, row id) of every row the program selects, written by the JIT scan -- the M_PART
    producer with one row-id field, then one split pass that compacts the chunk regions in order.
    Sketch aggregators that need the selected rows themselves (theta KMV) read these instead of a
    torch re-scan of the shard (``_rows`` + ``eval_bexpr`` + ``compute_keys``)."""

    def __init__(self, prog: ScanProgram):
        import copy

        from .lower import lds_layout

        ep = copy.copy(prog)
        ep.aops = [{"kind": D.A_ROWID, "col": -1, "expr": None, "filter": None, "slot": 0, "hll": -1}]
        ep.slots = [(D.S_SUM_I, 0)]
        ep.nhll, ep.stored_hll, ep.thetas, ep.packed = 0, [], [], {}
        ep.presence_only = False
        self.prog = ep
        self.dev = prog.ds.device
        from ..ops import jit as J

        if prog.empty or not J.part_eligible(ep) or J.part_hashed(ep):
            raise RuntimeError("emit: program not eligible")
        self.jit = _jit_for(ep, D.M_PART, False, 1 << prog.hll_p)
        if self.jit is None:
            raise RuntimeError("emit: no JIT kernel")
        cache_off, wave_bytes, _, total = lds_layout(ep, 0, UNROLL, BLOCK // 64)
        d = pack(ep, D.M_PART, 0, 0, 0, 0, 0, 0, 0, 0, 0, [], [], unroll=UNROLL, cache_off=cache_off,
                 wave_bytes=wave_bytes)
        self.nch = int(d[0]["total_chunks"])
        self.grid = _grid(self.dev, self.nch, self.jit.lay.total, self.jit)
        cap = self.nch * D.CHUNK_ROWS
        if 2 * cap >= (1 << 32):
            raise RuntimeError("emit: shard too large for u32 offsets")
        self.words = max(1, 2 * cap)
        self.seg_lo = (torch.arange(self.nch, dtype=torch.int64) * D.CHUNK_ROWS).to(torch.int32).to(self.dev)
        self.k = max(1, min(self.nch, 1024))
        self._d = d  # (host descriptor: each run uploads a copy naming its own record / offset buffers)

    def run(self):
        """(keys int64, rows int64) of the selected rows, in row order within each chunk.  The
        record buffers come from the shared partition-scratch pool and the small per-run state is
        allocated per run, so concurrent slots never share device state."""
        nat, st = native.load(), native._stream(self.dev)
        u32 = torch.int32
        pend = torch.empty(max(1, self.nch), dtype=u32, device=self.dev)
        counts = torch.empty(self.k, dtype=u32, device=self.dev)
        totals = torch.empty(1, dtype=u32, device=self.dev)
        base = torch.empty(2, dtype=u32, device=self.dev)
        slab = PART_POOL.acquire(self.dev, self.words)
        try:
            d = self._d.copy()
            d[0]["part_recs"] = slab.recs1.data_ptr()
            d[0]["part_counts"] = pend.data_ptr()
            desc = _upload(d.view(np.uint8), self.dev)
            nat.module_launch(self.jit.handle, desc.data_ptr(), int(self.grid), BLOCK, int(self.jit.lay.total), st)
            a = (slab.recs1.data_ptr(), 2, self.seg_lo.data_ptr(), pend.data_ptr(), 1, self.nch, self.k, 0, 1,
                 counts.data_ptr())
            nat.part_split(*a, 0, 0, 2, st)  # (one bucket: every wave adds once)
            nat.part_scan(counts.data_ptr(), 1, self.k, totals.data_ptr(), base.data_ptr(), st)
            nat.part_split(*a, base.data_ptr(), slab.recs2.data_ptr(), 3, st)
            n = int(base[1].item())
            rec = slab.recs2[: 2 * n].view(n, 2).to(torch.int64) & 0xFFFFFFFF
            return rec[:, 0].contiguous(), rec[:, 1].contiguous()
        finally:
            PART_POOL.release(slab)


def theta_producer_prog(prog: ScanProgram, cols: List[str]) -> ScanProgram:
    """The scan program of a fused theta producer: ``prog``'s filter, ranges and group key, one
    A_THETA aggregator (a 62-bit KMV hash, two record words) per theta column, no other aggregator.
    RuntimeError where it does not apply."""
    import copy

    from ..ops import jit as J

    ds = prog.ds
    for c in cols:
        m = ds.metrics.get(c)
        if c not in ds.dims and (m is None or m.sketch is not None or m.data.dtype.is_floating_point):
            raise RuntimeError("theta: fused only over dimension ids / integer metrics")
    ep = copy.copy(prog)
    ep.pcols, ep.fcols, ep.section = list(prog.pcols), list(prog.fcols), "p"
    ep.aops = [{"kind": D.A_THETA, "col": ep.col(c), "expr": None, "filter": None, "slot": i, "hll": -1}
               for i, c in enumerate(cols)]
    ep.slots = [(D.S_SUM_I, 0)] * len(cols)
    ep.nhll, ep.stored_hll, ep.thetas, ep.packed = 0, [], [], {}
    ep.presence_only = False
    if not J.part_eligible(ep) or J.part_hashed(ep):
        raise RuntimeError("theta: program not eligible")
    return ep


THETA_HIST_BINS = 2048


class PreparedTheta:
    """thetaSketch aggregators fused into the scan: ONE JIT producer pass (ops/jit.py A_THETA) writes
    (u32 group key, 62-bit KMV hash per theta column) records of the selected rows into its chunk
    regions, and the per-group radix select (ops/csrc/sketch.hip theta_*_regions: LDS histograms,
    bound, compaction) reads them in place -- no (key, row) pairs, no torch gather / hash of the
    selected rows, no compaction pass (round-4 SF10 7-group theta query: 29.5 ms).  Only the
    ~2k candidates per group reach the sort.  Query-time sketches over dimension ids and integer
    metrics (the hash input must equal ``column_tensor``'s value); G <= ``max_g``."""

    def __init__(self, prog: ScanProgram, cols: List[str], max_g: int):
        import copy

        from .lower import lds_layout
        from ..ops import jit as J

        ds = prog.ds
        if prog.empty or not (0 < prog.G <= max_g):
            raise RuntimeError("theta: program not eligible")
        ep = theta_producer_prog(prog, cols)
        self.prog, self.dev, self.G, self.nt = ep, ds.device, int(prog.G), len(cols)
        self.jit = _jit_for(ep, D.M_PART, False, 1 << prog.hll_p)
        if self.jit is None:
            raise RuntimeError("theta: no JIT kernel")
        cache_off, wave_bytes, _, total = lds_layout(ep, 0, UNROLL, BLOCK // 64)
        d = pack(ep, D.M_PART, 0, 0, 0, 0, 0, 0, 0, 0, 0, [], [], unroll=UNROLL, cache_off=cache_off,
                 wave_bytes=wave_bytes)
        self.nch = int(d[0]["total_chunks"])
        self.grid = _grid(self.dev, self.nch, self.jit.lay.total, self.jit)
        self.rw = 1 + 2 * self.nt
        cap = self.nch * D.CHUNK_ROWS
        if cap * self.rw >= (1 << 32):
            raise RuntimeError("theta: shard too large for u32 offsets")
        self.words = max(1, cap * self.rw)
        self.seg_lo = (torch.arange(self.nch, dtype=torch.int64) * D.CHUNK_ROWS).to(torch.int32).to(self.dev)
        self._d = d
        # histogram bits: few groups keep G x 2^bits <= THETA_HIST_BINS bins (every workgroup flushes
        # its nonzero bins with global atomics onto the same addresses: 4096 workgroups x 14K bins of
        # a 7-group SF10 query were 0.44 ms a pass); coarser bins only add candidates below the bound
        # (the filter keeps target + one bin's records).  Many groups: per-workgroup LDS [G][2^bits]
        # within 64 KiB when G allows, else 12 bits in global memory.
        gt = self.G * min(4, self.nt)  # (up to 4 sketches share one histogram pass: rows t * G + g)
        if gt <= THETA_HIST_BINS // 16:
            self.bits = int(math.floor(math.log2(THETA_HIST_BINS // gt)))
        else:
            fit = int(math.floor(math.log2(max(1, (64 * 1024 // 4) // gt))))
            self.bits = fit if fit >= 8 else 12
        self.bits = max(4, min(16, self.bits))
        # first-attempt target per aggregator, in multiples of 2k records: learnt from the previous
        # run (duplicate-heavy columns -- c_name repeats ~6x per ship mode -- need 4x-16x more records
        # than 2k below the bound for k distinct hashes; a repeated statement then selects in one pass)
        self._mult = {}
        self.attempts = {}  # (per aggregator: select passes of the last run)
        self._bounds = {}  # first sketch of a select group -> its last run's per-row bounds (device)

    def select(self, sizes: List[int], estimates: bool = False) -> list:
        """Per theta aggregator (``sizes``: its k) the sorted unique (group, hash) pairs of its k
        smallest distinct hashes per group -- or, with ``estimates`` (one rank: no union across
        ranks follows), the per-group theta estimates [G] as host float64 arrays, computed from the
        candidates directly: (k-1) / (h_k / 2^62), or the exact distinct count below k hashes
        (the same values engine/executor.py _kmv_estimates gives for the k-trimmed pairs)."""
        from .executor import _kmv, _sorted_unique_pairs

        nat, st = native.load(), native._stream(self.dev)
        pend = torch.empty(max(1, self.nch), dtype=torch.int32, device=self.dev)
        slab = PART_POOL.acquire(self.dev, self.words)
        out = []
        try:
            d = self._d.copy()
            d[0]["part_recs"] = slab.recs1.data_ptr()
            d[0]["part_counts"] = pend.data_ptr()
            desc = _upload(d.view(np.uint8), self.dev)
            nat.module_launch(self.jit.handle, desc.data_ptr(), int(self.grid), BLOCK, int(self.jit.lay.total), st)
            G, dev = self.G, self.dev
            # (host-side targets and capacities: the only syncs are the candidate count with the
            # largest bound after each filter pass, and the short-group check).  Up to 4 sketches
            # are selected together: one histogram and one filter pass over the records, candidate
            # groups t * G + g
            cap_all = max(1, self.nch * D.CHUNK_ROWS)
            out = [None] * len(sizes)
            for t0 in range(0, len(sizes), 4):
                ks = sizes[t0:t0 + 4]
                nt = len(ks)
                GT = G * nt
                hist = torch.empty(GT << self.bits, dtype=torch.int32, device=dev)
                bound = torch.empty(GT, dtype=torch.int64, device=dev)
                count = torch.zeros(1, dtype=torch.int64, device=dev)
                kk = np.repeat(np.asarray(ks, dtype=np.int64), G)  # k per row t * G + g
                mult = np.repeat(np.asarray([self._mult.get(t0 + j, 1) for j in range(nt)], dtype=np.int64), G)
                tgt = 2 * kk * mult
                cached = self._bounds.get(t0)
                for attempt in range(7):
                    # a repeated statement first filters with its last run's bounds (same rows, same
                    # candidates: no histogram pass); a short group falls back to the histogram
                    reuse = attempt == 0 and cached is not None
                    if reuse:
                        bound.copy_(torch.from_numpy(cached))
                    if attempt == 6:  # (never in practice after six 4x rounds): every pair
                        tgt = np.full(GT, 1 << 62, dtype=np.int64)
                    target = torch.from_numpy(tgt).to(dev)
                    cap = max(1, min(cap_all * nt, int(np.minimum(tgt, 1 << 40).sum()) * 2 + (1 << 16)))
                    while True:
                        og = torch.empty(cap, dtype=torch.int64, device=dev)
                        oh = torch.empty(cap, dtype=torch.int64, device=dev)
                        nat.theta_select_regions(slab.recs1.data_ptr(), self.rw, 1 + 2 * t0, self.seg_lo.data_ptr(),
                                                 pend.data_ptr(), self.nch, G, self.bits, hist.data_ptr(),
                                                 target.data_ptr(), bound.data_ptr(), og.data_ptr(), oh.data_ptr(),
                                                 count.data_ptr(), cap, st, nt, 1 if reuse else 0)
                        # (one copy: the candidate count, the largest bound, the bounds themselves --
                        # kept on the host for the next run, so no device tensor crosses streams)
                        vals = torch.cat([count.view(1), bound.max().view(1), bound]).cpu().numpy()
                        c, hmax = int(vals[0]), int(vals[1])
                        if c <= cap:
                            break
                        cap = c  # a duplicate-heavy bin held more candidates than the first guess
                    # (candidates are below their group's bound: one sort of g << s | h when they fit)
                    pairs = _sorted_unique_pairs(og[:c], oh[:c], GT, hmax)
                    distinct = torch.bincount(pairs[:, 0], minlength=GT) if pairs.numel() else \
                        torch.zeros(GT, dtype=torch.int64, device=dev)
                    short = ((distinct < torch.from_numpy(kk).to(dev)) & (bound < (1 << 62))).cpu().numpy()
                    if not short.any():
                        break
                    if reuse:
                        continue  # (the histogram path with this run's targets)
                    tgt = np.where(short, tgt * 4, tgt)
                    mult = np.where(short, np.minimum(mult * 4, 1 << 12), mult)
                self._bounds[t0] = vals[2:].copy()
                if estimates:
                    kt = torch.from_numpy(kk).to(dev)
                    first = torch.cumsum(distinct, 0) - distinct
                    kth_i = (first + torch.minimum(kt, distinct) - 1).clamp_(min=0)
                    kth = pairs[:, 1].index_select(0, kth_i.clamp_(max=max(0, pairs.shape[0] - 1))).to(torch.float64) \
                        if pairs.numel() else torch.zeros(GT, dtype=torch.float64, device=dev)
                    # (the same float expression, scalar k over the tensor, as _kmv_estimates: equal bits)
                    est = torch.cat([torch.where(distinct[j * G:(j + 1) * G] < ks[j],
                                                 distinct[j * G:(j + 1) * G].to(torch.float64),
                                                 (ks[j] - 1) / (kth[j * G:(j + 1) * G] / float(1 << 62)))
                                     for j in range(nt)]).cpu().numpy()
                    for j in range(nt):
                        self._mult[t0 + j] = int(mult[j * G:(j + 1) * G].max())
                        self.attempts[t0 + j] = attempt + 1
                        out[t0 + j] = est[j * G:(j + 1) * G]
                    continue
                # split the candidate rows t * G + g back into per-sketch (g, h) pairs (sorted by row)
                starts = torch.searchsorted(pairs[:, 0].contiguous(),
                                            torch.arange(nt + 1, device=dev, dtype=torch.int64) * G).tolist() \
                    if pairs.numel() else [0] * (nt + 1)
                for j in range(nt):
                    pj = pairs[starts[j]:starts[j + 1]]
                    if pj.numel():
                        pj = torch.stack([pj[:, 0] - j * G, pj[:, 1]], dim=1)
                    self._mult[t0 + j] = int(mult[j * G:(j + 1) * G].max())
                    self.attempts[t0 + j] = attempt + 1
                    out[t0 + j] = _kmv(pj, ks[j])
        finally:
            PART_POOL.release(slab)
        return out


class PreparedMask:
    """Filter-only scan: writes one u64 mask word per 64 rows (select queries); the mask becomes
    row ids with the ``compact_rows`` kernel (ops/csrc/post_scan.hip).  Mask + descriptor are
    per execution slot, like PreparedScan's buffers."""

    def __init__(self, prog: ScanProgram):
        import threading

        from .lower import lds_layout

        self.prog = prog
        self.dev = prog.ds.device
        cache_off, wave_bytes, _, total = lds_layout(prog, 0, UNROLL, BLOCK // 64)
        self._layout = (cache_off, wave_bytes)
        self.lds_total = total
        self.jit = _jit_for(prog, D.M_MASK, False, 2048) if not prog.empty else None
        self._slot_lock = threading.Lock()
        self._slots = {}
        self._bufs()

    def _bufs(self):
        slot = current_slot()
        b = self._slots.get(slot)
        if slot != 0:
            # the mask words come from the slot's arena (zeroed by every run); the descriptor is
            # re-packed only when the mask lands at another offset
            from .scheduler import slot_epoch

            ar = slot_arena(self.dev, slot)
            ep = slot_epoch(slot)
            if b is not None and b[3][0] == ar.gen and b[3][2] == ep:
                return b
            gen, off, _, buf = ar.carve(self.prog.ds.nwords * 8, self)
            if b is not None and b[3][:2] == (gen, off):
                b = (b[0], b[1], b[2], (gen, off, ep))
            else:
                mask = SlotArena.view(buf, off, self.prog.ds.nwords, torch.int64)
                b = self._make(mask) + ((gen, off, ep),)
            with self._slot_lock:
                self._slots[slot] = b
            return b
        if b is None:
            with self._slot_lock:
                b = self._slots.get(slot)
                if b is None:
                    mask = torch.zeros(self.prog.ds.nwords, dtype=torch.int64, device=self.dev)
                    b = self._slots[slot] = self._make(mask) + ((-1, -1, -1),)
        return b

    def _make(self, mask: torch.Tensor) -> tuple:
        prog = self.prog
        count = torch.zeros(1, dtype=torch.int64, device=self.dev)
        d = pack(prog, D.M_MASK, 0, 0, 0, 0, 0, 0, 0, mask.data_ptr(), count.data_ptr(), [], [],
                 unroll=UNROLL, cache_off=self._layout[0], wave_bytes=self._layout[1])
        desc = torch.from_numpy(d.view(np.uint8).copy()).to(self.dev)
        self.grid = _grid(self.dev, int(d[0]["total_chunks"]), self.jit.lay.total if self.jit else self.lds_total,
                          self.jit)
        return mask, count, desc

    def run(self) -> torch.Tensor:
        """Row ids passing the filter (sorted)."""
        if self.prog.empty:
            return torch.zeros(0, dtype=torch.int64, device=self.dev)
        mask, count, desc, _ = self._bufs()
        mask.zero_()
        count.zero_()
        if self.jit is not None:
            self.jit.launch(desc, self.grid)
        else:
            native.scan(desc, self.grid, BLOCK, self.lds_total, UNROLL)
        return native.compact_rows(mask)


PART_TABLE_BYTES = 32 << 10  # LDS table per sub-bucket
PART_MIN_SUBS = 512  # sub-buckets (aggregation workgroups) a partitioned group-by aims for at least
HASH_TABLE_BYTES = 128 << 10  # LDS hash table of a hash-partitioned sub-bucket (keys + slots)
PART_HLL_TABLE_BYTES = 128 << 10  # LDS slots + HLL byte registers of a partitioned sub-bucket
HLL32_MAX_BYTES = 512 << 20  # u32 scan-time registers


def part_layout(prog) -> dict:
    """Bucket geometry of the partitioned group-by for G keys: sub-buckets of 2^shift keys whose
    table (2^shift x nslots x 8 B) fits PART_TABLE_BYTES of LDS; the remaining key bits split
    over one level (<= 2^10 buckets) or two (level 1 <= 2^10 buckets, each split into P2 by K blocks)."""
    from ..ops import jit

    ns = max(1, prog.nslots)
    if jit.part_hashed(prog):
        return part_hash_layout(prog)
    nh = jit.part_hll_count(prog) if (prog.nhll or getattr(prog, "stored_hll", None)) else 0
    if nh:
        # a group's slots plus its byte registers: sub-buckets of a few dozen groups per LDS table
        per = 8 * ns + nh * (1 << prog.hll_p)
        shift = max(0, int(math.floor(math.log2(max(1, PART_HLL_TABLE_BYTES // per)))))
    else:
        shift = max(0, int(math.floor(math.log2(max(8, PART_TABLE_BYTES // (8 * ns))))))
    # enough sub-buckets to fill the chip: one aggregation workgroup per sub-bucket, so a key space
    # of a few thousand groups in 64 KiB tables (day x ship mode, 17.7K groups: 9 sub-buckets, 9
    # busy CUs, 11.6 ms at SF10) is cut into smaller tables instead
    shift = max(0, min(shift, int(math.floor(math.log2(max(1, prog.G // PART_MIN_SUBS))))))
    gbits = max(1, int(math.ceil(math.log2(max(2, prog.G)))))
    rem = max(0, gbits - shift)
    fields = jit.part_fields(prog)
    rw = 1 + sum(w for _, w in fields) + nh
    if rem <= 10:
        p1 = 1 << rem
        L = {"levels": 1, "shift": shift, "shift1": shift, "p1": p1, "p2": 1, "k": 1, "nsub": p1,
             "fields": fields, "rw": rw, "nhll": nh}
    else:
        b1 = min(10, (rem + 1) // 2)
        b2 = rem - b1
        if b2 > 10:
            raise ValueError(f"partitioned group-by: {prog.G} keys need more than two levels")
        p1, p2 = 1 << b1, 1 << b2
        k = max(1, min(64, 4096 // p1))
        L = {"levels": 2, "shift": shift, "shift1": shift + b2, "p1": p1, "p2": p2, "k": k, "nsub": p1 * p2,
             "fields": fields, "rw": rw, "nhll": nh}
    # (3+ word records only: one-word records stream at a third of the two-word rate through the
    # split and aggregation kernels -- TPC-H Q18 packed 2 -> 1 word was slower, profiles/r6/pack_ab.txt)
    pk = _pack_field(prog, fields, L["shift1"]) if PACK_RECORDS and not nh and rw >= 3 else None
    if pk is not None:
        j, word = pk
        L["pack"] = pk
        L["rw1"] = rw - 1
        L["agg_fields"] = [(s_, (3 | (L["shift1"] << 8)) if i == j else w_) for i, (s_, w_) in enumerate(fields)]
    return L


# The level-1 split packs one small non-negative value field of a partition record into the key
# word's bits above shift1 -- bits the level-1 bucket and the sub-bucket imply -- so the level-2
# split and the aggregation move one word less per record (the BI plan's TopVolumeCustomers: key +
# o_totalprice + l_quantity, 12 -> 8 bytes a record after level 1, 15.1 -> 12.6 ms a statement at
# SF100, tools/pack_ab.py, profiles/r6/pack_ab.txt).
PACK_RECORDS = True


def _value_range(ds, name: str):
    """(min, max) of a column's stored values (cached per datasource)."""
    cache = ds.__dict__.setdefault("_value_ranges", {})
    r = cache.get(name)
    if r is None:
        from .lower import column_tensor

        t = column_tensor(ds, name)
        if t.numel() == 0 or t.is_floating_point():
            r = cache[name] = False
        else:
            mn, mx = torch.aminmax(t)
            r = cache[name] = (int(mn), int(mx))
    return r or None


def _pack_field(prog, fields, shift1: int):
    """(field index, record word) of the first one-word field whose values fit the key word's bits
    above ``shift1``: a filtered count (0 / 1) or an unexpressioned integer sum over a column with
    non-negative values (a filter that rejects the row writes the identity 0).  None otherwise."""
    from ..ops import jit

    free = 32 - int(shift1)
    if free < 1 or not hasattr(prog, "aops"):
        return None
    cols = jit.col_infos(prog)
    by_slot = {a["slot"]: a for a in prog.aops}
    word = 1
    for j, (slot, wd) in enumerate(fields):
        if wd == 1:
            a = by_slot.get(slot)
            bits = None
            if a is not None and a["kind"] == D.A_COUNT and a.get("filt_len"):
                bits = 1
            elif a is not None and a["kind"] == D.A_SUM_I and not a.get("expr") and a.get("col") in cols:
                rng = _value_range(prog.ds, cols[a["col"]].name)
                if rng is not None and rng[0] >= 0:
                    bits = max(1, int(rng[1]).bit_length())
            if bits is not None and bits <= free:
                return j, word
        word += wd
    return None


def part_hash_layout(prog, scale: int = 1, groups: Optional[float] = None) -> dict:
    """Sub-buckets of a hash-partitioned group-by: enough that each holds ~half its LDS table's
    capacity of distinct keys by the group estimate -- the planner's row estimate at first, the
    observed group count once a run has seen it (``groups``) -- ``scale`` x more after an
    overflow; bucket bits are the top bits of the record's 32-bit hash, split over one level
    (<= 2^10 buckets) or two."""
    from ..ops import jit

    ns = max(1, prog.nslots)
    nh = jit.part_hll_count(prog) if (prog.nhll or getattr(prog, "stored_hll", None)) else 0
    per = 8 * (1 + ns) + nh * (1 << prog.hll_p)  # (a slot's key, slots and HLL byte registers)
    cap_log2 = max(6, min(14, int(math.floor(math.log2(max(1, HASH_TABLE_BYTES // per))))))
    if groups is None:
        groups = min(float(prog.G), float(getattr(prog, "est_rows", prog.G)) * 1.2)
    groups = max(1.0, groups)
    nsub = max(8, int(math.ceil(groups * scale / (1 << (cap_log2 - 1)))))
    bits = min(20, max(3, int(math.ceil(math.log2(nsub)))))
    fields = jit.part_fields(prog)
    rw = 3 + sum(w for _, w in fields) + nh
    if bits <= 10:
        p1 = 1 << bits
        return {"levels": 1, "hashed": True, "shift": 32 - bits, "shift1": 32 - bits, "p1": p1, "p2": 1, "k": 1,
                "nsub": p1, "fields": fields, "rw": rw, "cap_log2": cap_log2, "scale": scale, "nhll": nh}
    b1 = min(10, (bits + 1) // 2)
    b2 = bits - b1
    p1, p2 = 1 << b1, 1 << b2
    k = max(1, min(64, 4096 // p1))
    return {"levels": 2, "hashed": True, "shift": 32 - bits, "shift1": 32 - b1, "p1": p1, "p2": p2, "k": k,
            "nsub": p1 * p2, "fields": fields, "rw": rw, "cap_log2": cap_log2, "scale": scale, "nhll": nh}


def _grid(dev: torch.device, total_chunks: int, lds_total: int, jit=None) -> int:
    """Persistent grid: enough 8-wave blocks for the chunks, at most what the CUs hold at once --
    by LDS and, for a JIT kernel, by its compiled register use (the chunks are dealt to waves
    statically, so blocks beyond the resident set would run as a second, partial wave)."""
    waves = BLOCK // 64
    need = max(1, (total_chunks + waves - 1) // waves)
    per_cu = max(1, min(BLOCKS_PER_CU, (160 * 1024) // max(lds_total, 1)))
    if jit is not None:
        per_cu = max(1, min(per_cu, jit.occupancy()))
    return max(1, min(need, num_cus(dev) * per_cu))


_INIT_ROWS: dict = {}
_init_lock = threading.Lock()


def _init_row(dev, inits: tuple) -> torch.Tensor:
    """Device copy of a slot-init row, shared by every prepared scan with the same slots (read-only:
    the fused reset copies it into the accumulators)."""
    k = (str(dev), inits)
    t = _INIT_ROWS.get(k)
    if t is None:
        with _init_lock:
            t = _INIT_ROWS.get(k)
            if t is None:
                t = _upload(np.asarray(inits, dtype=np.int64).view(np.uint8), dev).view(torch.int64)
                if dev.type == "cuda":
                    torch.cuda.current_stream(dev).synchronize()  # (once: other streams read it)
                _INIT_ROWS[k] = t
    return t


def _upload(buf: np.ndarray, dev) -> torch.Tensor:
    """Host bytes -> a new device tensor without a synchronous pageable copy: staged through the
    caching pinned allocator and copied on the current stream (the staging block is not reused
    before that copy completes).  A statement first seen by a server allocates its descriptor this
    way on every slot; the pageable ``.to(dev)`` blocked the serving thread for each."""
    if dev.type != "cuda":
        return torch.from_numpy(buf.copy())
    h = torch.empty(buf.nbytes, dtype=torch.uint8, pin_memory=True)
    h.numpy()[:] = buf.reshape(-1)
    out = torch.empty(buf.nbytes, dtype=torch.uint8, device=dev)
    out.copy_(h, non_blocking=True)
    return out


def _nonzero_big(mask: torch.Tensor) -> torch.Tensor:
    """torch.nonzero in 2^30-element pieces (ROCm's nonzero miscounts past 2^31 elements: a hash
    table for 10^9 groups would ask for an absurd allocation)."""
    n = mask.numel()
    if n <= (1 << 30):
        return torch.nonzero(mask).flatten()
    step = 1 << 30
    return torch.cat([torch.nonzero(mask[a:a + step]).flatten() + a for a in range(0, n, step)])

