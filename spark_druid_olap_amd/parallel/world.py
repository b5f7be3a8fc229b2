"""Process-group abstraction: one process per GPU, torch.distributed over RCCL ("nccl" backend
on ROCm) for device tensors, gloo for CPU tests.

The reference scatters queries to Druid historicals over HTTP and merges on the broker or in a
Spark shuffle (``sd/DruidRDD.scala:62-99``, ``asd/PostAggregate.scala:97-103``); here every rank
owns a shard of every datasource in HBM and ranks merge partial aggregates with collectives
over xGMI (see ``parallel/merge.py``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    backend: str = "none"
    group: Any = None
    # a real process group of ONE rank whose collectives still run (``SDO_FORCE_COLLECTIVES=1``):
    # every distributed code path -- RCCL all-gather / all-to-all with splits / all-reduce / barrier
    # -- executes on a one-GPU box (tools/rccl_smoke.py, tests/test_gpu_rccl.py)
    force_collectives: bool = False

    @property
    def distributed(self) -> bool:
        return self.size > 1 or self.force_collectives

    @property
    def pg(self):
        """The process group this thread's collectives use: the SPMD server's per-slot group while
        a slot worker runs a statement (``slot_group``), else this world's group (default)."""
        g = getattr(_TLS, "group", None)
        return g if g is not None else self.group

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def device(self) -> torch.device:
        if torch.cuda.is_available() and (self.backend != "gloo" or _gloo_on_gpu()):
            return torch.device("cuda", self.local_rank % max(1, torch.cuda.device_count()))
        return torch.device("cpu")

    # gloo over device tensors (the one-GPU rehearsal of the multi-rank path: several ranks share
    # one card, which RCCL refuses): collectives stage through host memory.  RCCL takes device
    # tensors directly.
    def _stage(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if (t.is_cuda and self.backend == "gloo") else t

    def _unstage(self, h: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        if h is t:
            return t
        t.copy_(h)
        return t

    # ---------------------------------------------------------------- collectives
    def barrier(self):
        if self.distributed:
            _turn()
            if self.backend == "nccl":
                dist.barrier(group=self.pg, device_ids=[self.local_rank])
            else:
                dist.barrier(group=self.pg)

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if not self.distributed:
            return t
        _turn()
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        h = self._stage(t)
        dist.all_reduce(h, op=o, group=self.pg)
        return self._unstage(h, t)

    def all_gather_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """[size, *t.shape] stacked gather (same shape on every rank)."""
        return self.all_gather_tensor_async(t).wait()

    # Asynchronous forms: the collective is enqueued (RCCL: on the process group's own stream,
    # ordered after the work already on the current stream; gloo: on its worker thread) and
    # ``wait()`` returns the result (RCCL: the current stream waits for the collective, no host
    # sync).  Kernels launched in between -- the next segment batch's scan -- overlap it.
    def all_reduce_async(self, t: torch.Tensor, op: str = "sum") -> "Pending":
        if not self.distributed:
            return Pending(None, lambda: t)
        _turn()
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        h = self._stage(t)
        work = dist.all_reduce(h, op=o, group=self.pg, async_op=True)
        return Pending(work, lambda: self._unstage(h, t))

    def all_gather_tensor_async(self, t: torch.Tensor) -> "Pending":
        if not self.distributed:
            return Pending(None, lambda: t.unsqueeze(0))
        _turn()
        src = self._stage(t.contiguous().reshape(-1))
        # concatenated layout works on both RCCL and gloo (gloo rejects the stacked form)
        out = torch.empty((self.size * src.numel(),), dtype=t.dtype, device=src.device)
        work = dist.all_gather_into_tensor(out, src, group=self.pg, async_op=True)
        return Pending(work, lambda: out.to(t.device).view((self.size,) + tuple(t.shape)))

    def all_to_all_varlen(self, t: torch.Tensor, counts: torch.Tensor, status: Optional[int] = None):
        """Personalized exchange (the reference's hash-partitioned shuffle before the final
        aggregate, ``asd/PostAggregate.scala:97-103``): ``t``'s rows are grouped by destination rank
        (``counts[r]`` rows for rank r, in rank order); returns the rows every rank sent here,
        concatenated in source-rank order, plus the per-source counts.  One all-gather of the count
        vectors (carrying the status word, parallel/fault.py) and one ``all_to_all_single`` of the
        payload: each rank receives ~total/N rows instead of the all-gather's total.  With ``status`` set,
        ``(rows, recv_counts, statuses)`` is returned and a failure skips the payload exchange."""
        if not self.distributed:
            return (t, counts.clone(), [status]) if status is not None else (t, counts.clone())
        _turn()
        n = self.size
        dev = t.device
        # ONE host wait per exchange: every rank's whole send-count vector (and status word) is
        # all-gathered -- an [N, N + 1] matrix, on the device under RCCL, queued behind the kernels
        # that produced the counts -- and read back once.  Row r is what rank r sends, so this
        # rank's input splits (its own row) and output splits (its column) both come from the one
        # copy (a count exchange + a separate read of the local counts were two host round trips).
        mdev = counts.device if (self.backend == "nccl" and counts.is_cuda) else torch.device("cpu")
        send_meta = torch.cat([counts.to(device=mdev, dtype=torch.int64).reshape(-1),
                               torch.full((1,), int(status or 0), dtype=torch.int64, device=mdev)])
        send_meta = send_meta.to(dev if self.backend == "nccl" else "cpu").contiguous()
        recv_meta = torch.empty(n * (n + 1), dtype=torch.int64, device=send_meta.device)
        dist.all_gather_into_tensor(recv_meta, send_meta, group=self.pg)
        meta = recv_meta.reshape(n, n + 1).cpu()
        rc = meta[:, self.rank].clone()
        sent = meta[self.rank, :n].tolist()
        sts = meta[:, n].tolist()
        if status is not None and any(sts):
            return t[:0], rc, sts
        row = tuple(t.shape[1:])
        width = 1
        for x in row:
            width *= x
        src = self._stage(t.contiguous().reshape(-1))
        out = torch.empty((int(rc.sum()) * width,), dtype=t.dtype, device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=[int(x) * width for x in rc.tolist()],
                               input_split_sizes=[int(x) * width for x in sent], group=self.pg)
        out = out.to(dev).reshape((-1,) + row)
        return (out, rc, sts) if status is not None else (out, rc)

    def gather_varlen(self, t: torch.Tensor, root: int = 0, status: Optional[int] = None):
        """Rows of every rank concatenated at ``root`` only: an all-to-all in which each rank sends
        its rows to the root and nothing to anyone else, so the root takes in exactly the result
        (each peer over its own xGMI link) and no other rank receives a byte of it -- unlike an
        all-gather, which delivers N copies.  Returns ``(per-source tensors, statuses)``: the root
        gets one tensor per rank, the others an empty list; every rank learns every status (the
        count exchange carries it, parallel/fault.py)."""
        if not self.distributed:
            return [t], [status or 0]
        counts = torch.zeros(self.size, dtype=torch.int64)
        counts[root] = t.shape[0]
        out, rc, sts = self.all_to_all_varlen(t, counts, status=int(status or 0))
        if self.rank != root or any(sts):
            return [], sts
        return list(torch.split(out, [int(x) for x in rc.tolist()])), sts

    def all_gather_varlen(self, t: torch.Tensor, status: Optional[int] = None):
        """Gather tensors whose first dimension differs per rank.  With ``status`` set, every rank's
        status word rides along with the length exchange and ``(tensors, statuses)`` is returned
        (failure agreement without an extra collective, parallel/fault.py)."""
        if not self.distributed:
            return ([t], [status]) if status is not None else [t]
        n = torch.tensor([t.shape[0], status or 0], dtype=torch.int64, device=t.device)
        g = self.all_gather_tensor(n).reshape(self.size, 2).tolist()
        ns = [x[0] for x in g]
        sts = [x[1] for x in g]
        if status is not None and any(sts):
            return [t[:0]] * self.size, sts
        mx = max(ns) if ns else 0
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.shape[0]:
            pad[: t.shape[0]] = t
        g = self.all_gather_tensor(pad)
        out = [g[i, : ns[i]] for i in range(self.size)]
        return (out, sts) if status is not None else out

    def broadcast_object(self, obj: Any, src: int = 0, group=None) -> Any:
        """(``group``: a host-side (gloo) group of the same ranks -- the SPMD server's control
        stream, which then never occupies a GPU queue next to the statements' collectives)"""
        if not self.distributed:
            return obj
        if group is None:
            _turn()
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=group if group is not None else self.pg)
        return lst[0]

    def all_gather_object(self, obj: Any) -> List[Any]:
        """Small host metadata from every rank (catalog views, segment inventories)."""
        if not self.distributed:
            return [obj]
        _turn()
        out: List[Any] = [None] * self.size
        dist.all_gather_object(out, obj, group=self.pg)
        return out

    def max_float(self, x: float) -> float:
        if not self.distributed:
            return x
        dev = self.device() if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        # an all-gather, not a ring all-reduce: every rank talks to every peer, so a dead rank is
        # noticed by all survivors at once (parallel/recovery.py agrees on membership right after)
        return float(self.all_gather_tensor(t).max().item())


_TLS = __import__("threading").local()


# ------------------------------------------------------------------------------------------------
# Agreed issue order of collectives across concurrent statements (the SPMD server's execution slots,
# server/spmd.py).  Each slot has its own communicator, and RCCL enqueues a communicator's kernels on
# its own stream -- but a process has only GPU_MAX_HW_QUEUES (4) hardware queues for all of its
# streams.  If rank A enqueued slot 1's collective before slot 2's while rank B did the opposite,
# and the two landed on one in-order hardware queue on each rank, each rank's first kernel would
# spin waiting for a peer kernel queued behind the other one: a cross-communicator deadlock.  So
# every statement gets a sequence number in broadcast order (identical on every rank), and a thread
# running statement s issues a collective only once every statement before s has FINISHED: the
# collectives of all slots then leave every rank in the same order (statement by statement), and
# at most one statement is between collectives at a time.  Scans, compiles and host work of the
# slots still overlap freely; only their collective phases are ordered.
class IssueOrder:
    def __init__(self):
        import threading

        self.cv = threading.Condition()
        self.next_seq = 0
        self.active: set = set()
        self.log: Optional[list] = None  # (tests) the seq of every gated collective, in issue order

    def begin(self, seq: Optional[int] = None) -> int:
        """The next statement's sequence number (or the one the root assigned it) -- call in
        broadcast order on every rank."""
        with self.cv:
            s = self.next_seq if seq is None else int(seq)
            self.next_seq = max(self.next_seq, s + 1)
            self.active.add(s)
            return s

    def finish(self, seq: int) -> None:
        with self.cv:
            self.active.discard(seq)
            self.cv.notify_all()

    def wait_turn(self, seq: int, timeout_s: float = 3600.0) -> None:
        with self.cv:
            if not self.cv.wait_for(lambda: not self.active or min(self.active) >= seq, timeout=timeout_s):
                raise RuntimeError(f"statement {seq}: earlier statements {sorted(self.active)[:4]} never finished")
            if self.log is not None:
                self.log.append(seq)


class statement_turn:
    """``with statement_turn(order, seq):`` -- this thread runs statement ``seq``: its collectives
    wait for their turn (``IssueOrder``); the statement is finished on exit (``finish=False``: a
    part of the statement -- its preparation in the dispatch thread -- that is not the end of it)."""

    def __init__(self, order: Optional[IssueOrder], seq: Optional[int], finish: bool = True):
        self.order, self.seq, self.finish = order, seq, finish

    def __enter__(self):
        self._prev = (getattr(_TLS, "order", None), getattr(_TLS, "seq", None))
        _TLS.order, _TLS.seq = self.order, self.seq
        return self

    def __exit__(self, *exc):
        _TLS.order, _TLS.seq = self._prev
        if self.finish and self.order is not None and self.seq is not None:
            self.order.finish(self.seq)
        return False


def _turn() -> None:
    o = getattr(_TLS, "order", None)
    if o is not None:
        o.wait_turn(_TLS.seq)


class slot_group:
    """``with slot_group(g):`` -- collectives issued by this thread go to process group ``g``.

    The SPMD server runs K statements at once, one per execution slot, each slot with its own
    process group created identically on every rank (``dist.new_group``): statements of different
    slots then issue their collectives concurrently on independent communicators, while within a
    slot every rank issues them in the same (broadcast) order."""

    def __init__(self, group):
        self.group = group

    def __enter__(self):
        self._prev = getattr(_TLS, "group", None)
        _TLS.group = self.group
        return self

    def __exit__(self, *exc):
        _TLS.group = self._prev
        return False


class Pending:
    """An enqueued collective; ``wait()`` returns its result."""
    __slots__ = ("work", "_result")

    def __init__(self, work, result):
        self.work = work
        self._result = result

    def wait(self):
        if self.work is not None:
            self.work.wait()
        return self._result()


_WORLD: Optional[World] = None


def _gloo_on_gpu() -> bool:
    """``SDO_GLOO_GPU=1``: ranks keep their shards on the GPU but talk over gloo (several ranks on
    one card -- a rehearsal of the multi-GPU code paths on a one-GPU box)."""
    return os.environ.get("SDO_GLOO_GPU", "0") not in ("0", "")


def init_world(backend: Optional[str] = None, timeout_s: int = 600) -> World:
    """Initialise from torchrun env vars (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*)."""
    global _WORLD
    size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    forced = size <= 1 and os.environ.get("SDO_FORCE_COLLECTIVES", "0") not in ("0", "")
    if size <= 1 and not forced:
        _WORLD = World(0, 1, local, "none")
        return _WORLD
    size = max(1, size)
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() and not _gloo_on_gpu() else "gloo"
    if backend == "gloo" and _gloo_on_gpu() and torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    if backend == "nccl":
        torch.cuda.set_device(local % torch.cuda.device_count())
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local % torch.cuda.device_count())
        timeout_s = int(os.environ.get("SDO_COLLECTIVE_TIMEOUT_S", timeout_s))
        dist.init_process_group(backend=backend, rank=rank, world_size=size,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _WORLD = World(rank, size, local, backend, None, force_collectives=forced)
    return _WORLD


def get_world() -> World:
    global _WORLD
    if _WORLD is None:
        if dist.is_available() and dist.is_initialized():
            b = dist.get_backend()
            _WORLD = World(dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", dist.get_rank())), b)
        else:
            _WORLD = World()
    return _WORLD


def set_world(w: World) -> None:
    global _WORLD
    _WORLD = w


def shutdown() -> None:
    global _WORLD
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _WORLD = None
