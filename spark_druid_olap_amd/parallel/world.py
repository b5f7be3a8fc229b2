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

    @property
    def distributed(self) -> bool:
        return self.size > 1

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
            if self.backend == "nccl":
                dist.barrier(group=self.pg, device_ids=[self.local_rank])
            else:
                dist.barrier(group=self.pg)

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if not self.distributed:
            return t
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
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        h = self._stage(t)
        work = dist.all_reduce(h, op=o, group=self.pg, async_op=True)
        return Pending(work, lambda: self._unstage(h, t))

    def all_gather_tensor_async(self, t: torch.Tensor) -> "Pending":
        if not self.distributed:
            return Pending(None, lambda: t.unsqueeze(0))
        src = self._stage(t.contiguous().reshape(-1))
        # concatenated layout works on both RCCL and gloo (gloo rejects the stacked form)
        out = torch.empty((self.size * src.numel(),), dtype=t.dtype, device=src.device)
        work = dist.all_gather_into_tensor(out, src, group=self.pg, async_op=True)
        return Pending(work, lambda: out.to(t.device).view((self.size,) + tuple(t.shape)))

    def all_to_all_varlen(self, t: torch.Tensor, counts: torch.Tensor, status: Optional[int] = None):
        """Personalized exchange (the reference's hash-partitioned shuffle before the final
        aggregate, ``asd/PostAggregate.scala:97-103``): ``t``'s rows are grouped by destination rank
        (``counts[r]`` rows for rank r, in rank order); returns the rows every rank sent here,
        concatenated in source-rank order, plus the per-source counts.  One ``all_to_all_single`` of
        the counts (carrying the status word, parallel/fault.py) and one of the payload: each rank
        receives ~total/N rows instead of the all-gather's total.  With ``status`` set,
        ``(rows, recv_counts, statuses)`` is returned and a failure skips the payload exchange."""
        if not self.distributed:
            return (t, counts.clone(), [status]) if status is not None else (t, counts.clone())
        n = self.size
        dev = t.device
        # (RCCL: the counts stay on the device -- the meta exchange is queued behind the kernels
        # that produced them, and the one host wait is for the received meta below)
        mdev = counts.device if (self.backend == "nccl" and counts.is_cuda) else torch.device("cpu")
        send_meta = torch.stack([counts.to(device=mdev, dtype=torch.int64),
                                 torch.full((n,), int(status or 0), dtype=torch.int64, device=mdev)], 1)
        send_meta = send_meta.to(dev if self.backend == "nccl" else "cpu").reshape(-1).contiguous()
        recv_meta = torch.empty_like(send_meta)
        dist.all_to_all_single(recv_meta, send_meta, group=self.pg)
        meta = recv_meta.reshape(n, 2).cpu()
        rc = meta[:, 0]
        sts = meta[:, 1].tolist()
        if status is not None and any(sts):
            return t[:0], rc, sts
        row = tuple(t.shape[1:])
        width = 1
        for x in row:
            width *= x
        src = self._stage(t.contiguous().reshape(-1))
        out = torch.empty((int(rc.sum()) * width,), dtype=t.dtype, device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=[int(x) * width for x in rc.tolist()],
                               input_split_sizes=[int(x) * width for x in counts.cpu().tolist()], group=self.pg)
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

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.distributed:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.pg)
        return lst[0]

    def all_gather_object(self, obj: Any) -> List[Any]:
        """Small host metadata from every rank (catalog views, segment inventories)."""
        if not self.distributed:
            return [obj]
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
    if size <= 1:
        _WORLD = World(0, 1, local, "none")
        return _WORLD
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
    _WORLD = World(rank, size, local, backend, None)
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
