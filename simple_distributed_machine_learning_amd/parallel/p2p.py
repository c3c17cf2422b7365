"""Transport seam: every cross-rank byte the engine moves goes through one of these objects.

Replaces the reference's RRef hand-off (``RRef(z3)`` + ``rpc_sync().forward`` + ``to_here()``,
/root/reference/simple_distributed.py:47-49, :71), the Send/Recv autograd functions of
distributed autograd (:112) and the optimizer RPCs (:113). The engine never calls
``torch.distributed`` itself; it asks its :class:`Transport` for

* ``isend`` / ``irecv``  point-to-point boundary tensors (classic neighbour pipelines),
* ``all_to_all``         a wave's stage boundary fanned out over every peer (``rotate``),
* ``all_reduce``         data-parallel gradient sums, tensor-parallel partial sums, metrics,
* ``barrier``.

Two implementations are interchangeable behind that interface ("one small
transport seam"):

* :class:`DirectTransport` hands the tensors to ``torch.distributed`` as they are: RCCL over
  xGMI for device tensors (``Work.wait()`` is a stream-level wait, nothing blocks the host),
  Gloo over loopback for CPU tensors (the CPU test path).
* :class:`HostStagedTransport` moves DEVICE tensors through host memory over Gloo: device ->
  host copy, Gloo op, host -> device copy on the consumer's stream. RCCL refuses two ranks on
  one GPU, so this is what lets a 1-GPU box run 2..16 ranks of the real device engine (every
  kernel, every orchestration branch of the R > 1 paths) in separate processes sharing
  ``cuda:0`` (``SDML_TRANSPORT=host``; tests/test_multirank_gpu.py).

:class:`BufferPool` holds the persistent boundary buffers: one per (role, slot), sized on first
use and reused by every later step, so the step loop allocates no communication memory.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def message_tag(payload: int, pipe: int, stage: int, mb: int) -> int:
    return (((mb * 4096 + stage) * 2 + pipe) * 2 + payload) & 0x3FFFFFFF


class _Done:
    """A completed operation (nothing to wait for)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


class BufferPool:
    """Persistent device buffers keyed by (role, slot).

    ``get(key, shape, dtype)`` returns a view of the buffer for ``key``, allocated on first use
    (or when a larger shape / other dtype is asked for) and reused afterwards. A step uses each key
    at most once, and every consumer of a buffer is stream-ordered before the next step's producer
    (RCCL waits for the compute stream when a collective is enqueued), so reuse across steps is
    safe without host synchronisation. ``allocations`` counts real allocations (tests assert it
    stops growing after the first step).

    ``retain``: set once a HIP graph has been captured over these buffers (parallel/graphs.py). A graph
    keeps raw addresses, not tensor references, so a buffer replaced by a larger one must stay alive
    while a graph may replay into it: replaced buffers then move to ``_retired`` instead of going back
    to the allocator."""

    def __init__(self, device: torch.device):
        self.device = device
        self._bufs: Dict[tuple, torch.Tensor] = {}
        self._retired = []
        self.retain = False
        self.allocations = 0

    def get(self, key: tuple, shape: Sequence[int], dtype: torch.dtype) -> torch.Tensor:
        shape = tuple(int(s) for s in shape)
        n = math.prod(shape)
        buf = self._bufs.get(key)
        if buf is None or buf.dtype != dtype or buf.numel() < n:
            if buf is not None and self.retain:
                self._retired.append(buf)
            buf = torch.empty(max(n, 1), dtype=dtype, device=self.device)
            self._bufs[key] = buf
            self.allocations += 1
        return buf[:n].view(shape)

    def nbytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in self._bufs.values())


class Transport:
    """Interface + byte accounting shared by the implementations."""

    name = "base"

    def __init__(self, mesh):
        self.mesh = mesh
        self._pending_sends: List[tuple] = []
        self.bytes_sent = 0   # bytes this rank put on links (all_to_all: other ranks' parts only)
        self.bytes_recv = 0
        self.ops = 0

    # ---- group selection -------------------------------------------------------------------
    def _p2p_group(self, src: int, dst: int):
        g = self.mesh.p2p_groups.get((src, dst))
        if g is None:
            raise RuntimeError(f"no p2p channel {src}->{dst} (ranks must be pipeline neighbours)")
        return g

    def _channel(self, channel: str):
        m = self.mesh
        if channel == "fwd":
            return m.pipe_group
        if channel == "bwd":
            return m.pipe_group_bwd or m.pipe_group
        if channel == "grad":
            return m.grad_group
        if channel == "world":
            return None
        raise ValueError(f"unknown transport channel {channel!r}")

    def _count_a2a(self, out_splits, in_splits, row_bytes):
        me = self.mesh.pp_rank
        self.bytes_sent += row_bytes * (sum(in_splits) - in_splits[me])
        self.bytes_recv += row_bytes * (sum(out_splits) - out_splits[me])

    # ---- operations (implemented below) ----------------------------------------------------
    def isend(self, t: torch.Tensor, dst: int, tag: int):
        raise NotImplementedError

    def irecv(self, t: torch.Tensor, src: int, tag: int):
        raise NotImplementedError

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Sequence[int],
                   in_splits: Sequence[int], channel: str = "fwd"):
        raise NotImplementedError

    def all_reduce(self, t: torch.Tensor, group=None, channel: Optional[str] = None, op=dist.ReduceOp.SUM,
                   async_op: bool = True):
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def drain_sends(self):
        """Wait for all outstanding sends (end of step; keeps their buffers alive until then)."""
        for w, _ in self._pending_sends:
            w.wait()
        self._pending_sends.clear()

    def reset_counters(self):
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.ops = 0


class DirectTransport(Transport):
    """``torch.distributed`` on the tensors themselves: RCCL (device) or Gloo (CPU)."""

    name = "direct"

    def __init__(self, mesh):
        super().__init__(mesh)
        self.use_tags = mesh.backend != "nccl"

    def isend(self, t, dst, tag):
        t = t.contiguous()
        w = dist.isend(t, dst, group=self._p2p_group(self.mesh.rank, dst), tag=tag if self.use_tags else 0)
        self._pending_sends.append((w, t))
        self.bytes_sent += t.numel() * t.element_size()
        self.ops += 1
        return w

    def irecv(self, t, src, tag):
        w = dist.irecv(t, src, group=self._p2p_group(src, self.mesh.rank), tag=tag if self.use_tags else 0)
        self.bytes_recv += t.numel() * t.element_size()
        self.ops += 1
        return w

    def all_to_all(self, out, inp, out_splits, in_splits, channel="fwd"):
        row = (inp[0].numel() if inp.dim() > 1 else 1) * inp.element_size() if inp.numel() else 0
        self._count_a2a(out_splits, in_splits, row)
        self.ops += 1
        return dist.all_to_all_single(out, inp.contiguous(), list(out_splits), list(in_splits),
                                      group=self._channel(channel), async_op=True)

    def all_reduce(self, t, group=None, channel=None, op=dist.ReduceOp.SUM, async_op=True):
        g = group if channel is None else self._channel(channel)
        self.ops += 1
        w = dist.all_reduce(t, op=op, group=g, async_op=async_op)
        return w if async_op else _Done()

    def barrier(self):
        if self.mesh.backend == "nccl" and self.mesh.device.type == "cuda":
            dist.barrier(device_ids=[self.mesh.device.index])
        else:
            dist.barrier()


class _StagedWork:
    """A Gloo operation on a host copy; ``wait()`` finishes it and moves the result to the device
    tensor on the caller's current stream (the consumer's stream, as with RCCL)."""

    def __init__(self, work, host: Optional[torch.Tensor], dev: Optional[torch.Tensor]):
        self.work, self.host, self.dev = work, host, dev
        self._done = False

    def wait(self):
        if not self._done:
            self.work.wait()
            if self.dev is not None and self.dev.numel():
                self.dev.copy_(self.host.view_as(self.dev))
            self._done = True
        return True

    def is_completed(self):
        return self._done


class HostStagedTransport(Transport):
    """Device tensors through host memory over Gloo (multi-rank on one GPU; slow but exact: the
    bytes delivered are the bytes sent)."""

    name = "host"

    @staticmethod
    def _host(t: torch.Tensor) -> torch.Tensor:
        return t.detach().contiguous().to("cpu")  # synchronous: the producer kernel has finished

    def isend(self, t, dst, tag):
        h = self._host(t)
        w = dist.isend(h, dst, group=self._p2p_group(self.mesh.rank, dst), tag=tag)
        self._pending_sends.append((w, h))
        self.bytes_sent += t.numel() * t.element_size()
        self.ops += 1
        return w

    def irecv(self, t, src, tag):
        h = torch.empty(t.shape, dtype=t.dtype)
        w = dist.irecv(h, src, group=self._p2p_group(src, self.mesh.rank), tag=tag)
        self.bytes_recv += t.numel() * t.element_size()
        self.ops += 1
        return _StagedWork(w, h, t)

    def all_to_all(self, out, inp, out_splits, in_splits, channel="fwd"):
        row = (inp[0].numel() if inp.dim() > 1 else 1) * inp.element_size() if inp.numel() else 0
        self._count_a2a(out_splits, in_splits, row)
        self.ops += 1
        hin = self._host(inp)
        hout = torch.empty(out.shape, dtype=out.dtype)
        w = dist.all_to_all_single(hout, hin, list(out_splits), list(in_splits), group=self._channel(channel),
                                   async_op=True)
        sw = _StagedWork(w, hout, out)
        sw._keep = hin
        return sw

    def all_reduce(self, t, group=None, channel=None, op=dist.ReduceOp.SUM, async_op=True):
        g = group if channel is None else self._channel(channel)
        self.ops += 1
        if t.device.type == "cpu":
            w = dist.all_reduce(t, op=op, group=g, async_op=async_op)
            return w if async_op else _Done()
        h = self._host(t)
        w = _StagedWork(dist.all_reduce(h, op=op, group=g, async_op=True), h, t)
        if not async_op:
            w.wait()
        return w

    def barrier(self):
        dist.barrier()


TRANSPORTS = {"direct": DirectTransport, "host": HostStagedTransport}


def make_transport(mesh) -> Transport:
    try:
        cls = TRANSPORTS[mesh.transport_kind]
    except KeyError:
        raise ValueError(f"unknown transport {mesh.transport_kind!r} (choose from {sorted(TRANSPORTS)})") from None
    return cls(mesh)
