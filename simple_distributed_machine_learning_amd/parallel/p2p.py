"""Point-to-point transport seam: activations forward, gradients backward.

Replaces the reference's RRef hand-off (``RRef(z3)`` + ``rpc_sync().forward`` + ``to_here()``,
/root/reference/simple_distributed.py:47-49, :71) and the Send/Recv autograd functions of
distributed autograd (:112). Here the producer *pushes* with ``isend`` right after the
producing kernel, the consumer posts ``irecv`` into a pre-allocated buffer, and only the
consumer's compute stream waits on the receive (``Work.wait()`` is a stream-level wait on
RCCL, not a host block), so transfers overlap with compute.

One channel (process group) per ordered rank pair: with RCCL each is its own communicator
+ HIP stream, i.e. an independent FIFO over the direct xGMI link between the two GPUs.
With Gloo (CPU tests) the same calls run over TCP loopback; tags keep messages apart.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .mesh import Mesh


def message_tag(payload: int, pipe: int, stage: int, mb: int) -> int:
    return (((mb * 4096 + stage) * 2 + pipe) * 2 + payload) & 0x3FFFFFFF


class Transport:
    def __init__(self, mesh: Mesh):
        self.mesh = mesh
        self._pending_sends: List[dist.Work] = []
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.use_tags = mesh.backend != "nccl"

    def _group(self, src: int, dst: int):
        g = self.mesh.p2p_groups.get((src, dst))
        if g is None:
            raise RuntimeError(f"no p2p channel {src}->{dst} (ranks must be pipeline neighbours)")
        return g

    def isend(self, t: torch.Tensor, dst: int, tag: int) -> dist.Work:
        t = t.contiguous()
        w = dist.isend(t, dst, group=self._group(self.mesh.rank, dst), tag=tag if self.use_tags else 0)
        self._pending_sends.append((w, t))
        self.bytes_sent += t.numel() * t.element_size()
        return w

    def irecv(self, t: torch.Tensor, src: int, tag: int) -> dist.Work:
        w = dist.irecv(t, src, group=self._group(src, self.mesh.rank), tag=tag if self.use_tags else 0)
        self.bytes_recv += t.numel() * t.element_size()
        return w

    def drain_sends(self):
        """Wait for all outstanding sends (end of step; keeps buffers alive until then)."""
        for w, _ in self._pending_sends:
            w.wait()
        self._pending_sends.clear()

    def reset_counters(self):
        self.bytes_sent = 0
        self.bytes_recv = 0
