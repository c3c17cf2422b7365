"""Flat parameter / gradient / momentum storage for all stages a rank owns.

Every parameter of the rank's stage modules becomes a view into ONE contiguous fp32 (or the
model dtype) buffer; ``.grad`` views point into a second buffer. Consequences on MI355X:

* the optimizer is one fused HIP launch over the whole buffer (ops/optim.py),
* the data-parallel gradient sync is one (or a few, bucketed) RCCL all-reduce(s) over a
  contiguous region — no per-tensor launches, no gather/scatter copies,
* zeroing gradients is one memset.

Offsets are padded to 64 elements (256 B) so every view starts 16-B aligned for
vectorised kernels. The order is (stage id, parameter registration order) so replicas of
the same stage set on different ranks (DP replicas, Chimera mirrors) line up element-wise.

The reference instead gathers per-parameter RRefs across processes
(/root/reference/simple_distributed.py:52-58, :82-83) for its DistributedOptimizer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn as nn

ALIGN = 64


def _pad(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class Segment:
    stage: int
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]


class FlatParams:
    def __init__(self, modules: Sequence[Tuple[int, nn.Module]], device, dtype=torch.float32):
        """modules: (stage_id, module) pairs; duplicates of the same stage id are not allowed."""
        mods = sorted(modules, key=lambda x: x[0])
        ids = [s for s, _ in mods]
        if len(set(ids)) != len(ids):
            raise ValueError("FlatParams: duplicate stage ids")
        self.segments: List[Segment] = []
        self.stage_ranges: Dict[int, Tuple[int, int]] = {}
        off = 0
        plist = []
        padded = []
        for sid, m in mods:
            start = off
            # a module may ask for zero rows after a 2-D parameter (flat_row_multiple = {name: multiple}): the rows
            # up to the next multiple stay zero in the parameter, gradient, master and momentum buffers (their
            # gradient is zero, so SGD keeps them zero), so a kernel may treat the weight as the padded
            # [rows rounded up][cols] matrix in place (ops/linear.py lm_head: GPT-2's 50257-row vocabulary -> 50304)
            mult = getattr(m, "flat_row_multiple", None) or {}
            for name, p in m.named_parameters():
                self.segments.append(Segment(sid, name, off, p.numel(), tuple(p.shape)))
                plist.append(p)
                n = p.numel()
                if name in mult and p.dim() == 2:
                    rows = -(-p.shape[0] // mult[name]) * mult[name]
                    n = rows * p.shape[1]
                    padded.append((p, rows))
                off += _pad(n)
            self.stage_ranges[sid] = (start, off)
        self.numel = max(off, ALIGN)
        self.device = torch.device(device)
        self.dtype = dtype
        self.params = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.grads = torch.zeros(self.numel, device=self.device, dtype=dtype)
        for seg, p in zip(self.segments, plist):
            view = self.params[seg.offset:seg.offset + seg.numel].view(seg.shape)
            view.copy_(p.detach().to(self.device, dtype))
            p.data = view
            p.grad = self.grads[seg.offset:seg.offset + seg.numel].view(seg.shape)
        for p, rows in padded:
            p._sdml_rows_padded = rows  # the storage holds `rows` rows (params and grads); the extra rows are zero
        self._plist = plist
        self.grads_zero = True  # grads known to be all-zero (skip the next zero_grad launch)
        # bumped by every optimizer step (whose kernels write the parameters through raw pointers,
        # which torch's per-tensor version counters do not see); with ``param._version`` it
        # identifies the parameter values a derived cache (ops.PlaneCache) was computed from
        self.param_epoch = 0

    def zero_grad(self, force: bool = False):
        if force or not self.grads_zero:
            self.grads.zero_()
        self.grads_zero = True

    def stage_slice(self, stage: int, which: str = "grads") -> torch.Tensor:
        a, b = self.stage_ranges[stage]
        return getattr(self, which)[a:b]

    def rebind_grads(self):
        """Re-point ``.grad`` at the flat buffer (call if something replaced a .grad)."""
        for seg, p in zip(self.segments, self._plist):
            g = self.grads[seg.offset:seg.offset + seg.numel].view(seg.shape)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g

    def check_bound(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() ==
                   self.grads[s.offset:s.offset + s.numel].data_ptr()
                   for s, p in zip(self.segments, self._plist))
