"""Peer-to-peer one-shot merge of small dense partials over IPC-mapped mailboxes.

The RCCL path for a small dense state is an ``all_gather_into_tensor``, one torch reduction per
slot and a host read of the status words: several launches and a host round trip per query, on
queries whose whole scan takes 0.1-0.4 ms at SF100.  Here every process group gets, once, one
device mailbox per rank (``ops/csrc/p2p.hip``): each rank exports its mailbox with an IPC handle,
the handles travel in one ``all_gather_object`` on that group, and every rank maps every peer's
mailbox.  A merge is then ONE kernel per rank that publishes its partial, waits for the peers'
(system-scope flags, bounded by a timeout) and reduces them with the per-slot operators -- peers
read over their own xGMI links (or, for ranks sharing one card in the rehearsal, through the same
device memory).  The status words come back next to the merged state; ``finalize`` checks them
together with the result's device-to-host copy instead of a separate host read.

Enabled when every rank's partials live on a GPU, the group has at most 8 ranks and every rank
could map every peer's mailbox (agreed collectively when the exchange is built); RCCL stays the
path for large and sparse states (``planner/cost.py plan_merge``).  ``SDO_P2P_MERGE=0`` disables it.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional, Tuple

import torch

P2P_MAX_BYTES = 64 << 10     # per-rank state (accumulator words + HLL register bytes + status)
HEADER = 256
MAX_RANKS = 8
MAX_SLOTS = 64
TIMEOUT_S = float(os.environ.get("SDO_P2P_TIMEOUT_S", "30"))
ENABLED = os.environ.get("SDO_P2P_MERGE", "1") != "0"

_lock = threading.Lock()
_EXCHANGES: Dict[Tuple, Optional["PeerExchange"]] = {}
_KEY_LOCKS: Dict[Tuple, threading.Lock] = {}


class PeerExchange:
    """Mailboxes of one process group: this rank's own (allocated here) and every peer's (mapped)."""

    def __init__(self, world, dev: torch.device):
        from ..ops import native

        nat = native.load()
        self.nat = nat
        self.rank, self.size = world.rank, world.size
        self.slot_bytes = P2P_MAX_BYTES
        own, handle = 0, None
        try:
            with torch.cuda.device(dev):
                own, handle = nat.p2p_alloc(HEADER + 2 * self.slot_bytes)
        except Exception:  # noqa: BLE001  (no IPC export here: agreed below, every rank falls back)
            pass
        self.own = own
        # (every step below is collective whatever happened locally, so no rank is left waiting)
        got = world.all_gather_object((world.rank, handle))
        mbox: List[int] = [0] * self.size
        ok = all(h is not None for _, h in got)
        opened = []
        with torch.cuda.device(dev):
            for r, h in got:
                if not ok:
                    break
                if r == world.rank:
                    mbox[r] = own
                    continue
                try:
                    mbox[r] = nat.p2p_open(h)
                    opened.append(mbox[r])
                except Exception:  # noqa: BLE001  (agreed below: every rank falls back together)
                    ok = False
        # every rank must have mapped every peer, or nobody uses the exchange
        self.ok = all(world.all_gather_object(ok))
        self.mbox = mbox
        self._opened = opened
        self.epoch = 0

    def merge(self, prog, part, status: int):
        """(merged Partials with ``status_dev`` = every rank's status word) -- enqueued on the
        current stream, no host synchronisation."""
        from ..engine.partials import Partials

        acc = part.acc.contiguous()
        R, ns = acc.shape
        hll = [h if h.dtype == torch.uint8 else h.clamp(0, 255).to(torch.uint8) for h in part.hll]
        flat = torch.cat([h.reshape(-1) for h in hll]) if hll else torch.zeros(0, dtype=torch.uint8, device=acc.device)
        pad = (-flat.numel()) % 8
        if pad:
            flat = torch.cat([flat, torch.zeros(pad, dtype=torch.uint8, device=flat.device)])
        flat = flat.contiguous()
        out_acc = torch.empty_like(acc)
        out_hll = torch.empty_like(flat)
        sts = torch.empty(self.size, dtype=torch.int64, device=acc.device)
        self.epoch += 1
        ops = [int(op) for op, _ in prog.slots]
        self.nat.p2p_merge(self.mbox, self.rank, self.epoch, self.slot_bytes, acc.data_ptr(), acc.numel(),
                           flat.data_ptr() if flat.numel() else acc.data_ptr(), flat.numel(), ops, int(status),
                           out_acc.data_ptr(), out_hll.data_ptr() if flat.numel() else out_acc.data_ptr(),
                           sts.data_ptr(), TIMEOUT_S, torch.cuda.current_stream(acc.device).cuda_stream)
        regs, off = [], 0
        for h in hll:
            n = h.numel()
            regs.append(out_hll[off: off + n].view(h.shape))
            off += n
        merged = Partials("dense", out_acc, None, regs)
        merged.status_dev = sts
        merged.status_rank = self.rank
        return merged

    def close(self) -> None:
        for p in self._opened:
            self.nat.p2p_close(p)
        self._opened = []
        if self.own:
            self.nat.p2p_free(self.own)
            self.own = 0


def fits(prog, part) -> bool:
    """Layout-only test (identical on every rank): the state fits a mailbox slot and the kernel."""
    if part.kind != "dense" or not part.acc.is_cuda or prog.nslots < 1 or prog.nslots > MAX_SLOTS:
        return False
    hll = sum(h.numel() for h in part.hll)
    return part.acc.numel() * 8 + (hll + 7) // 8 * 8 + 8 <= P2P_MAX_BYTES


def exchange_for(world) -> Optional[PeerExchange]:
    """The exchange of the calling thread's process group (built collectively on first use: every
    rank reaches a group's first small dense merge at the same point of the same statement)."""
    if not ENABLED or not world.distributed or world.size > MAX_RANKS or not torch.cuda.is_available():
        return None
    dev = world.device()
    if dev.type != "cuda":
        return None
    key = (id(world.pg), world.rank, str(dev))
    ex = _EXCHANGES.get(key, False)
    if ex is not False:
        return ex
    # one lock per group: building an exchange is a collective on that group, and two slot groups
    # building theirs at once on different threads must not wait on each other
    with _lock:
        klock = _KEY_LOCKS.setdefault(key, threading.Lock())
    with klock:
        ex = _EXCHANGES.get(key, False)
        if ex is False:
            ex = PeerExchange(world, dev)
            if not ex.ok:
                ex.close()
                ex = None
            _EXCHANGES[key] = ex
    return ex


def check_status(part) -> None:
    """Host check of a P2P merge's status words (for consumers that do not fetch them with the
    result copy)."""
    sts = getattr(part, "status_dev", None)
    if sts is None:
        return
    from .fault import raise_if_failed

    part.status_dev = None
    vals = sts.tolist()
    if any(vals):
        raise_if_failed(vals, part.status_rank, None)


def reset() -> None:
    with _lock:
        for ex in _EXCHANGES.values():
            if ex is not None:
                ex.close()
        _EXCHANGES.clear()


__all__ = ["PeerExchange", "exchange_for", "fits", "check_status", "P2P_MAX_BYTES"]
