"""Peer-to-peer one-shot merge of small dense partials over IPC-mapped mailboxes.

The RCCL path for a small dense state is an ``all_gather_into_tensor``, one torch reduction per
slot and a host read of the status words: several launches and a host round trip per query, on
queries whose whole scan takes 0.1-0.4 ms at SF100.  Here the main process group gets, once, one
device mailbox per rank (``ops/csrc/p2p.hip``, uncached device memory): each rank exports its
mailbox with an IPC handle, the handles travel in one ``all_gather_object``, and every rank maps
every peer's mailbox.  A merge is then ONE kernel per rank that publishes its partial, waits for the
peers' (system-scope flags) and reduces them with the per-slot operators -- peers read over their
own xGMI links (or, for ranks sharing one card in the rehearsal, through the same device memory).
The status words come back next to the merged state; ``finalize`` checks them together with the
result's device-to-host copy instead of a separate host read.

Fail-safe by construction:

* **Known-value self-test.**  When the exchange is built, every rank merges a state whose answer it
  knows (rank ids over both mailbox parities) and checks the result; the exchange is used only if
  every rank's check passed (agreed collectively), else every rank stays on RCCL.
* **Agreed retry.**  The kernel's wait for the peers' partials is bounded by a SOFT timeout
  (``SDO_P2P_TIMEOUT_S``, 0.5 s).  A rank that gives up posts that verdict; every rank reads every
  verdict, so all of them report ``STATUS_P2P_RETRY`` together, ``finalize`` / ``check_status``
  raise ``P2PRetry`` on every rank, and the statement re-runs with the merge over RCCL
  (``PreparedQuery``).  After ``MAX_RETRIES`` consecutive such epochs the group stops using the
  exchange (every rank counts the same epochs).  Only a peer that posts no verdict within the HARD
  timeout (a dead process, or a live one later than that deadline: the early rank then publishes
  an aborted final word, so every rank reports the timeout) turns into a failed status word.
* **One exchange per rank.**  Only statements on the main process group use it: SPMD execution
  slots (``server/spmd.py``) each have their own group and stream, and spinning merge kernels of
  different slots could share one hardware queue in a different order on different ranks.

Enabled when every rank's partials live on a GPU and the group has at most 8 ranks; RCCL stays the
path for large and sparse states (``planner/cost.py plan_merge``).  ``SDO_P2P_MERGE=0`` disables it.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from typing import Dict, List, Optional, Tuple

import torch

P2P_MAX_BYTES = 64 << 10     # per-rank state (accumulator words + HLL register bytes + status)
HEADER = 256
MAX_RANKS = 8
MAX_SLOTS = 64
SOFT_TIMEOUT_S = float(os.environ.get("SDO_P2P_TIMEOUT_S", "0.5"))
HARD_TIMEOUT_S = float(os.environ.get("SDO_P2P_HARD_TIMEOUT_S", "10"))
MAX_RETRIES = 3
ENABLED = os.environ.get("SDO_P2P_MERGE", "1") != "0"


def _hook(name: str) -> Dict[str, float]:
    spec = os.environ.get(name, "")
    return {k: float(v) for k, v in (x.split("=", 1) for x in spec.split(",") if "=" in x)}


# test hooks: SDO_P2P_SELFTEST_FAIL=<rank> fails that rank's self-test check;
# SDO_P2P_DELAY="rank=1,s=1.5,times=1" delays that rank's merge launches (a peer's soft wait expires)
SELFTEST_FAIL_RANK = int(os.environ.get("SDO_P2P_SELFTEST_FAIL", "-1"))
DELAY = _hook("SDO_P2P_DELAY")

_lock = threading.Lock()
_EXCHANGES: Dict[Tuple, Optional["PeerExchange"]] = {}
_KEY_LOCKS: Dict[Tuple, threading.Lock] = {}
_TLS = threading.local()


class _SelfTestProg:
    def __init__(self):
        from ..ops import desc as D

        self.slots = [(D.S_SUM_I, 0), (D.S_MAX_I, -(1 << 62))]
        self.nslots = 2


class PeerExchange:
    """Mailboxes of one process group: this rank's own (allocated here) and every peer's (mapped)."""

    def __init__(self, world, dev: torch.device):
        from ..ops import native

        nat = native.load()
        self.nat = nat
        self.rank, self.size = world.rank, world.size
        self.slot_bytes = P2P_MAX_BYTES
        own, handle, self.memory = 0, None, None
        try:
            with torch.cuda.device(dev):
                own, handle, self.memory = nat.p2p_alloc(HEADER + 2 * self.slot_bytes)
        except Exception:  # noqa: BLE001  (no IPC export here: agreed below, every rank falls back)
            pass
        self.own = own
        self.dev = dev
        self.retries = 0        # consecutive abandoned epochs (reset by a completed one)
        self.total_retries = 0
        self.disabled = False
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
        self.selftest = None
        if self.ok:
            # known values over both mailbox parities; used only if every rank's check passed
            try:
                self.selftest = self._self_test()
            except Exception as e:  # noqa: BLE001  (agreed below)
                self.selftest = f"error: {e}"
            self.ok = all(world.all_gather_object(self.selftest is True))

    def _self_test(self):
        """Each rank contributes (rank + 1) * [[1, 10], [2, -1]] (int sum, int max) and HLL bytes
        with rank + 1 at position ``rank``; every rank must read back the exact merge of all N,
        with every status word clean, in two consecutive epochs (both data slots)."""
        from ..engine.partials import Partials

        n, r = self.size, self.rank
        prog = _SelfTestProg()
        want_acc = [[n * (n + 1) // 2, 10 * n], [n * (n + 1), -1]]
        want_hll = [i + 1 if i < n else 0 for i in range(16)]
        for epoch in range(2):
            acc = torch.tensor([[r + 1, 10 * (r + 1)], [2 * (r + 1), -(r + 1)]], dtype=torch.int64, device=self.dev)
            hll = torch.zeros((1, 16), dtype=torch.uint8, device=self.dev)
            hll[0, r] = r + 1
            m = self.merge(prog, Partials("dense", acc, None, [hll]), 0, soft_s=max(SOFT_TIMEOUT_S, 2.0))
            sts = m.status_dev.tolist()
            got_acc, got_hll = m.acc.tolist(), m.hll[0].reshape(-1).tolist()
            if SELFTEST_FAIL_RANK == r:
                got_acc = [[0, 0], [0, 0]]
            if any(sts) or got_acc != want_acc or got_hll != want_hll:
                return f"epoch {epoch}: status {sts}, acc {got_acc} (want {want_acc}), hll {got_hll}"
        return True

    def merge(self, prog, part, status: int, soft_s: Optional[float] = None):
        """(merged Partials with ``status_dev`` = every rank's status word) -- enqueued on the
        current stream, no host synchronisation."""
        from ..engine.partials import Partials

        if DELAY and int(DELAY.get("rank", -1)) == self.rank and DELAY.get("times", 1) > 0 and self.epoch >= 2:
            DELAY["times"] = DELAY.get("times", 1) - 1
            time.sleep(DELAY.get("s", 1.0))  # (test hook: after the self-test's two epochs)
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
                           sts.data_ptr(), float(soft_s if soft_s is not None else SOFT_TIMEOUT_S), HARD_TIMEOUT_S,
                           torch.cuda.current_stream(acc.device).cuda_stream)
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


def _key(world):
    return (id(world.pg), world.rank, str(world.device()))


@contextlib.contextmanager
def suppressed():
    """``with suppressed():`` -- merges issued by this thread take the RCCL path (the retry of a
    statement whose P2P epoch was abandoned)."""
    prev = getattr(_TLS, "off", False)
    _TLS.off = True
    try:
        yield
    finally:
        _TLS.off = prev


def exchange_for(world) -> Optional[PeerExchange]:
    """The exchange of the main process group (built collectively on first use: every rank reaches
    the group's first small dense merge at the same point of the same statement)."""
    from .world import _TLS as _WTLS

    if not ENABLED or not world.distributed or world.size > MAX_RANKS or not torch.cuda.is_available():
        return None
    if getattr(_TLS, "off", False) or getattr(_WTLS, "group", None) is not None:
        return None  # (a retry over RCCL, or an SPMD execution slot's own group)
    dev = world.device()
    if dev.type != "cuda":
        return None
    key = (id(world.pg), world.rank, str(dev))
    ex = _EXCHANGES.get(key, False)
    if ex is False:
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
    if ex is None or ex.disabled:
        return None
    return ex


def note_retry(world) -> None:
    """A statement's P2P epoch was abandoned (every rank calls this for the same epochs): after
    ``MAX_RETRIES`` of them the group's merges stay on RCCL."""
    ex = _EXCHANGES.get(_key(world))
    if ex:
        ex.retries += 1
        ex.total_retries += 1
        if ex.retries >= MAX_RETRIES:
            ex.disabled = True


def stats(world) -> Dict[str, object]:
    ex = _EXCHANGES.get(_key(world), False)
    if ex is False:
        return {"built": False}
    if ex is None:
        return {"built": True, "enabled": False}
    return {"built": True, "enabled": not ex.disabled, "memory": ex.memory, "epochs": ex.epoch,
            "retries": ex.retries, "total_retries": ex.total_retries, "selftest": ex.selftest}


def check_status(part) -> None:
    """Host check of a P2P merge's status words (for consumers that do not fetch them with the
    result copy).  Raises ``P2PRetry`` (every rank together) or ``RankFailure``."""
    sts = getattr(part, "status_dev", None)
    if sts is None:
        return
    part.status_dev = None
    raise_status(sts.tolist(), part.status_rank)


def note_ok(rank: int) -> None:
    """A completed epoch (every rank reads the same verdicts, so every rank resets together):
    ``MAX_RETRIES`` counts CONSECUTIVE abandoned epochs -- a few slow statements over a long run do
    not switch the exchange off for good."""
    for ex in _EXCHANGES.values():
        if ex is not None and ex.rank == rank and ex.retries:
            ex.retries = 0


def raise_status(vals: List[int], rank: int) -> None:
    from .fault import STATUS_P2P_TIMEOUT, raise_if_failed

    if not any(vals):
        note_ok(rank)
        return
    if any(vals):
        if any(int(v) == STATUS_P2P_TIMEOUT for v in vals):
            # a peer missed the hard deadline: this rank's epochs may no longer line up with it
            for ex in _EXCHANGES.values():
                if ex is not None and ex.rank == rank:
                    ex.disabled = True
        raise_if_failed(vals, rank, None)


def reset() -> None:
    with _lock:
        for ex in _EXCHANGES.values():
            if ex is not None:
                ex.close()
        _EXCHANGES.clear()


__all__ = ["PeerExchange", "exchange_for", "fits", "check_status", "raise_status", "note_retry", "suppressed",
           "stats", "P2P_MAX_BYTES"]
