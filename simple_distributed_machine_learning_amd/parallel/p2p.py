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
* :class:`IpcTransport` moves point-to-point boundary tensors DEVICE to DEVICE between processes:
  persistent send slots exported once as hipIPC memory handles, ordered on the device by stream
  memory operations (``hipStreamWriteValue32`` / ``hipStreamWaitValue32``), no host round trip
  (``SDML_TRANSPORT=ipc``; SURVEY.md §2c "hipIPC peer-write fast path with pre-registered
  persistent buffers"), the rotate placement's all-to-alls over the same pairwise channels, and the
  gradient all-reduce over the mapped flat-gradient slices.

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


class _IpcRecv:
    """An irecv of the IPC transport: ``wait()`` enqueues, on the caller's current stream, the wait for the sender's
    ready word, the copy out of the sender's slot and the acknowledgement (nothing blocks the host once the slot is
    mapped). ``parts``: several such receives completed by one ``wait()`` (the all-to-all)."""

    def __init__(self, tr, parts):
        self.tr, self.parts = tr, parts
        self._done = False

    def wait(self):
        if not self._done:
            for src, chan, t, seq in self.parts:
                self.tr._consume(src, chan, t, seq)
            self._done = True
        return True

    def is_completed(self):
        return self._done


class IpcTransport(HostStagedTransport):
    """Device tensors between processes through hipIPC: point-to-point boundary tensors, the rotate placement's
    all-to-alls and the data-parallel gradient all-reduce (other all-reduces stay host-staged). Exercised with
    processes sharing one GPU (the 1-GPU pool); between GPUs of a node the same handles need peer access.

    Per ordered channel (src -> dst, stream name) the SENDER owns ``SLOTS`` persistent slot buffers and one control
    block of int32 words: ``ready[s]`` (the sequence number of the last message written into slot s) and ``ack[s]``
    (the last one the receiver copied out). Both are exported once as IPC memory handles through the job's rendezvous
    store and opened once by the receiver. Messages on a channel are FIFO (the schedule matches every send with a recv
    in order; an all-to-all is one message per peer on its own stream name), so message k of a channel uses slot
    (k - 1) % SLOTS on both sides and nothing but the payload travels per message:

    * ``isend`` (sender's current stream): wait until ``ack[s] >= k - SLOTS`` (the slot's previous message was taken),
      copy the tensor into the slot, write ``ready[s] = k``;
    * ``irecv(...).wait()`` (receiver's current stream): wait until ``ready[s] >= k``, copy the slot into the tensor,
      write ``ack[s] = k``.

    Slot buffers come in power-of-two capacity classes (>= 64 KiB) that both sides derive from the message size, so
    a ragged last batch uses its own buffer without any negotiation. The words are written and waited on by the
    streams' command processors (hipStreamWriteValue32 / hipStreamWaitValue32 in ``_kernels``), so the hand-off is
    ordered on the device like an RCCL send / recv. The reference's hand-off this replaces is ``RRef(z3)`` +
    ``rpc_sync().forward`` + ``to_here()`` (/root/reference/simple_distributed.py:47-49, :71) and the gradient's way
    back (:112)."""

    name = "ipc"
    SLOTS = 16
    MIN_CLASS = 1 << 16
    _instances = 0  # per process; every rank builds its transports in the same order (SPMD), so the ids match

    def __init__(self, mesh):
        super().__init__(mesh)
        if mesh.device.type != "cuda":
            raise ValueError("the IPC transport moves device tensors: it needs a ROCm device")
        IpcTransport._instances += 1
        self.prefix = f"sdml_ipc/{IpcTransport._instances}"
        self.store = dist.distributed_c10d._get_default_store()
        self._send_seq: Dict[tuple, int] = {}
        self._recv_seq: Dict[tuple, int] = {}
        self._send_ctrl: Dict[tuple, torch.Tensor] = {}
        self._recv_ctrl: Dict[tuple, torch.Tensor] = {}
        self._send_bufs: Dict[tuple, torch.Tensor] = {}
        self._recv_bufs: Dict[tuple, torch.Tensor] = {}
        self._group_ranks: Dict[str, List[int]] = {}
        self._ar_reg: Dict[tuple, dict] = {}
        self._ar_ctrl = None
        self._ar_seq = 0
        self.registered = 0  # buffers exported (sender side) + opened (receiver side): tests assert it stops growing
        from .._native import kernels

        self.k = kernels()

    # ---- registration (once per channel / slot / capacity class) ------------------------------------------------
    def _key(self, src, dst, chan, what):
        return f"{self.prefix}/{src}->{dst}/{chan}/{what}"

    def _export(self, key, t):
        import pickle

        from torch.multiprocessing.reductions import reduce_tensor

        self.store.set(key, pickle.dumps(reduce_tensor(t)))
        self.registered += 1

    def _open(self, key):
        import pickle

        fn, args = pickle.loads(self.store.get(key))  # blocks until the peer has exported it (store timeout)
        self.registered += 1
        return fn(*args)

    @classmethod
    def _cls(cls, nbytes):
        return max(cls.MIN_CLASS, 1 << max(0, int(nbytes - 1).bit_length()))

    def _ctrl_out(self, dst, chan):
        c = self._send_ctrl.get((dst, chan))
        if c is None:
            c = self._send_ctrl[(dst, chan)] = torch.zeros(2 * self.SLOTS, dtype=torch.int32, device=self.mesh.device)
            torch.cuda.synchronize(self.mesh.device)  # zeroed before the peer can map it
            self._export(self._key(self.mesh.rank, dst, chan, "ctrl"), c)
        return c

    def _ctrl_in(self, src, chan):
        c = self._recv_ctrl.get((src, chan))
        if c is None:
            c = self._recv_ctrl[(src, chan)] = self._open(self._key(src, self.mesh.rank, chan, "ctrl"))
        return c

    def _slot_out(self, dst, chan, slot, cls):
        b = self._send_bufs.get((dst, chan, slot, cls))
        if b is None:
            b = self._send_bufs[(dst, chan, slot, cls)] = torch.empty(cls, dtype=torch.uint8, device=self.mesh.device)
            self._export(self._key(self.mesh.rank, dst, chan, f"s{slot}c{cls}"), b)
        return b

    def _slot_in(self, src, chan, slot, cls):
        b = self._recv_bufs.get((src, chan, slot, cls))
        if b is None:
            b = self._recv_bufs[(src, chan, slot, cls)] = self._open(self._key(src, self.mesh.rank, chan,
                                                                               f"s{slot}c{cls}"))
        return b

    @staticmethod
    def _bytes(t):
        return t.reshape(-1).view(torch.uint8)

    # ---- point to point ------------------------------------------------------------------------------------------
    def _send(self, t, dst, chan):
        t = t.detach().contiguous()
        n = t.numel() * t.element_size()
        k = self._send_seq.get((dst, chan), 0) + 1
        self._send_seq[(dst, chan)] = k
        slot = (k - 1) % self.SLOTS
        ctrl = self._ctrl_out(dst, chan)
        buf = self._slot_out(dst, chan, slot, self._cls(n))
        if k > self.SLOTS:  # the receiver has copied out this slot's previous message
            self.k.stream_wait_value32(ctrl.data_ptr() + 4 * (self.SLOTS + slot), k - self.SLOTS)
        if n:
            buf[:n].copy_(self._bytes(t))
        self.k.stream_write_value32(ctrl.data_ptr() + 4 * slot, k)
        return n

    def _post_recv(self, src, chan, t):
        k = self._recv_seq.get((src, chan), 0) + 1
        self._recv_seq[(src, chan)] = k
        return (src, chan, t, k)

    def isend(self, t, dst, tag):
        self.bytes_sent += self._send(t, dst, "p2p")
        self.ops += 1
        return _Done()

    def irecv(self, t, src, tag):
        self.bytes_recv += t.numel() * t.element_size()
        self.ops += 1
        return _IpcRecv(self, [self._post_recv(src, "p2p", t)])

    def _consume(self, src, chan, t, k):
        n = t.numel() * t.element_size()
        slot = (k - 1) % self.SLOTS
        ctrl = self._ctrl_in(src, chan)
        buf = self._slot_in(src, chan, slot, self._cls(n))
        self.k.stream_wait_value32(ctrl.data_ptr() + 4 * slot, k)
        if n:
            if t.is_contiguous():
                self._bytes(t).copy_(buf[:n])
            else:
                t.copy_(buf[:n].view(t.dtype).view(t.shape))
        self.k.stream_write_value32(ctrl.data_ptr() + 4 * (self.SLOTS + slot), k)

    # ---- all-to-all over the pairwise channels ---------------------------------------------------------------------
    def _ranks(self, channel):
        r = self._group_ranks.get(channel)
        if r is None:
            g = self._channel(channel)
            r = self._group_ranks[channel] = (list(range(dist.get_world_size())) if g is None
                                              else dist.get_process_group_ranks(g))
        return r

    def all_to_all(self, out, inp, out_splits, in_splits, channel="fwd"):
        """``out`` gets out_splits[j] rows from group member j, member j gets in_splits[j] rows of ``inp`` (the
        torch all_to_all_single contract, first dimension split): one message per peer on stream name
        ``a2a-<channel>``, the own part copied locally; ``wait()`` consumes the peers' parts on the caller's stream."""
        row = (inp[0].numel() if inp.dim() > 1 else 1) * inp.element_size() if inp.numel() else 0
        self._count_a2a(out_splits, in_splits, row)
        self.ops += 1
        ranks = self._ranks(channel)
        me = self.mesh.rank
        chan = f"a2a-{channel}"
        io = [0]
        for s in in_splits:
            io.append(io[-1] + int(s))
        oo = [0]
        for s in out_splits:
            oo.append(oo[-1] + int(s))
        parts = []
        for j, r in enumerate(ranks):
            src_part, dst_part = inp[io[j]:io[j + 1]], out[oo[j]:oo[j + 1]]
            if r == me:
                if dst_part.numel():
                    dst_part.copy_(src_part)
                continue
            self._send(src_part, r, chan)
            parts.append(self._post_recv(r, chan, dst_part))
        return _IpcRecv(self, parts)

    # ---- gradient all-reduce over the mapped buffers -------------------------------------------------------------
    def all_reduce(self, t, group=None, channel=None, op=dist.ReduceOp.SUM, async_op=True):
        """The data-parallel gradient sum (channel "grad": slices of the persistent flat gradient buffer) device to
        device: every member maps every other member's buffer once (registered in call order, which is the same on
        every rank), then per call, on the caller's stream: publish ``ready`` = k, wait for every member's ``ready``,
        sum the members' buffers in rank order into a temporary (the same bits on every rank), publish ``done`` = k,
        wait for every member's ``done`` (nobody still reads this buffer), copy the sum back. Other all-reduces
        (metrics, tensor-parallel partial sums on fresh tensors, MIN / MAX) stay host-staged."""
        if (channel != "grad" or op != dist.ReduceOp.SUM or t.device.type != "cuda" or not t.is_contiguous()
                or t.numel() == 0):
            return super().all_reduce(t, group=group, channel=channel, op=op, async_op=async_op)
        ranks = self._ranks("grad")
        me = self.mesh.rank
        self.ops += 1
        key = (t.data_ptr(), t.numel(), t.dtype)
        reg = self._ar_reg.get(key)
        if reg is None:  # first use of this buffer: export it, map every member's (same registration index)
            idx = len(self._ar_reg)
            self._export(self._key(me, "all", "ar", f"b{idx}"), t)
            peers = {r: (t if r == me else self._open(self._key(r, "all", "ar", f"b{idx}"))) for r in ranks}
            reg = self._ar_reg[key] = peers
        if self._ar_ctrl is None:  # [ready, done] words per member
            c = torch.zeros(2, dtype=torch.int32, device=self.mesh.device)
            torch.cuda.synchronize(self.mesh.device)
            self._export(self._key(me, "all", "ar", "ctrl"), c)
            self._ar_ctrl = {r: (c if r == me else self._open(self._key(r, "all", "ar", "ctrl"))) for r in ranks}
        self._ar_seq += 1
        k = self._ar_seq
        ctrl = self._ar_ctrl
        self.k.stream_write_value32(ctrl[me].data_ptr(), k)
        for r in ranks:
            if r != me:
                self.k.stream_wait_value32(ctrl[r].data_ptr(), k)
        acc = reg[ranks[0]].clone()
        for r in ranks[1:]:
            acc.add_(reg[r])
        self.k.stream_write_value32(ctrl[me].data_ptr() + 4, k)
        for r in ranks:
            if r != me:
                self.k.stream_wait_value32(ctrl[r].data_ptr() + 4, k)
        t.copy_(acc)  # (bytes_sent counts boundary tensors only, as in the other transports)
        return _Done()

    def drain_sends(self):
        self._pending_sends.clear()  # (sends are stream-ordered device copies: nothing to wait for on the host)


TRANSPORTS = {"direct": DirectTransport, "host": HostStagedTransport, "ipc": IpcTransport}


def make_transport(mesh) -> Transport:
    try:
        cls = TRANSPORTS[mesh.transport_kind]
    except KeyError:
        raise ValueError(f"unknown transport {mesh.transport_kind!r} (choose from {sorted(TRANSPORTS)})") from None
    return cls(mesh)
