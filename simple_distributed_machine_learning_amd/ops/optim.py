"""Per-stage fused SGD with momentum over the rank's flat parameter buffer.

Replaces ``DistributedOptimizer(optim.SGD, param_rrefs, lr=0.1, momentum=0.5)``
(/root/reference/simple_distributed.py:100-104, :113), which creates one TorchScript
``_FunctionalSGD`` per parameter owner and drives each step by RPC. Here each rank updates
the parameters it owns with ONE kernel launch over its flat buffer (utils/flat.py); the
update rule is torch.optim.SGD's (dampening 0, no nesterov, no weight decay by default):
``buf = momentum * buf + g`` (``buf = g`` on the first step), ``p -= lr * buf``.
"""
from __future__ import annotations

import os

import torch

from . import sgd_momentum_, sgd_momentum_mixed_
from ..utils.flat import FlatParams


class FusedSGD:
    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.flat = flat
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        # low-precision models (bf16 GPT-2) keep fp32 master weights + fp32 momentum here
        self.master = flat.params.float().clone() if flat.params.dtype != torch.float32 else None
        ref = self.master if self.master is not None else flat.params
        self.momentum_buffer = torch.zeros_like(ref) if momentum != 0 else ref.new_zeros(64)
        self.steps = 0
        self.plane_cache = None  # (PlaneCache, weight, flat offset): written by the step kernel

    def add_plane_cache(self, cache, weight: torch.Tensor) -> bool:
        """Have the fp32 step kernel also write ``cache`` (ops.PlaneCache) from ``weight``'s updated
        values. One cache per optimizer (the kernel takes one); returns False if not taken."""
        if self.master is not None or self.plane_cache is not None or not self.flat.params.is_cuda:
            return False
        off = (weight.data_ptr() - self.flat.params.data_ptr()) // self.flat.params.element_size()
        if not (0 <= off < self.flat.numel) or off % 4 or weight.shape[1] % 4:
            return False
        self.plane_cache = (cache, weight, off)
        return True

    def step(self, zero_grad: bool = True):
        """One update. ``zero_grad`` clears the gradients inside the same kernel (the engine
        then skips its own zero_grad at the next step: one launch, one pass over memory)."""
        if self.master is not None:
            sgd_momentum_mixed_(self.master, self.flat.params, self.flat.grads, self.momentum_buffer, self.lr,
                                self.momentum, self.dampening, self.weight_decay, self.nesterov, self.steps == 0,
                                zero_grad)
        else:
            planes = None
            if self.plane_cache is not None:
                cache, w, off = self.plane_cache
                planes = (cache.planes, off, w.shape[0], w.shape[1])
            sgd_momentum_(self.flat.params, self.flat.grads, self.momentum_buffer, self.lr, self.momentum,
                          self.dampening, self.weight_decay, self.nesterov, self.steps == 0, zero_grad, planes)
        if zero_grad:
            self.flat.grads_zero = True
        self.steps += 1
        self.flat.param_epoch += 1
        _weights_rewritten()
        if self.plane_cache is not None:
            from . import PlaneCache

            cache, w, _ = self.plane_cache
            cache.token = PlaneCache.token_of(w, self.flat.param_epoch)

    def fused_args(self, spans, zero_grad: bool = True):
        """Arguments for applying this optimizer's step inside the reduction that produces the step's
        last gradients (ops.linear_wgrad_u8_dl ``sgd``), or None when that cannot cover the whole step:
        ``spans`` = [(first grad tensor, numel)] of the flat gradient ranges that reduction writes;
        every parameter segment must lie inside them (the padding between segments stays zero)."""
        if self.master is not None or not self.flat.params.is_cuda or os.environ.get("SDML_FUSED_STEP", "1") == "0":
            return None
        base, es = self.flat.grads.data_ptr(), self.flat.grads.element_size()
        ranges = [((t.data_ptr() - base) // es, n) for t, n in spans]
        for seg in self.flat.segments:
            if not any(o <= seg.offset and seg.offset + seg.numel <= o + n for o, n in ranges):
                return None
        planes, poff, prows, pk = None, 0, 0, 0
        if self.plane_cache is not None:
            cache, w, poff = self.plane_cache
            planes, prows, pk = cache.planes, w.shape[0], w.shape[1]
        return (self.flat.params, self.flat.grads, self.momentum_buffer, float(self.lr), float(self.momentum),
                float(self.dampening), float(self.weight_decay), bool(self.nesterov), self.steps == 0,
                bool(zero_grad), planes, int(poff), int(prows), int(pk))

    def commit_fused(self, zero_grad: bool = True, planes_current: bool = True):
        """Book-keeping of a step that a fused kernel applied (what step() does after its kernel):
        ``fused_args``' reductions, or the whole-step kernel (``planes_current=False``: it did not
        write the weight-plane cache, which the next uint8 forward then re-splits)."""
        if zero_grad:
            self.flat.grads_zero = True
        self.steps += 1
        self.flat.param_epoch += 1
        _weights_rewritten()
        if self.plane_cache is not None:
            from . import PlaneCache

            cache, w, _ = self.plane_cache
            cache.token = PlaneCache.token_of(w, self.flat.param_epoch) if planes_current else None

    def buffer_view(self, param: torch.Tensor):
        """The momentum buffer's view aligned with ``param`` (a view into the flat parameter buffer), or
        None without momentum."""
        if self.momentum == 0:
            return None
        off = (param.data_ptr() - self.flat.params.data_ptr()) // self.flat.params.element_size()
        return self.momentum_buffer[off:off + param.numel()].view(param.shape)

    def zero_grad(self):
        self.flat.zero_grad()

    # ---- checkpoint (per-parameter names, reference-compatible keys) ----------------------
    def state_dict_for_stage(self, stage: int) -> dict:
        bufs = {}
        for seg in self.flat.segments:
            if seg.stage == stage and self.momentum != 0:
                bufs[seg.name] = self.momentum_buffer[seg.offset:seg.offset + seg.numel].view(seg.shape).detach().cpu().clone()
        out = {"momentum_buffer": bufs, "steps": self.steps, "lr": self.lr, "momentum": self.momentum,
               "dampening": self.dampening, "weight_decay": self.weight_decay, "nesterov": self.nesterov}
        if self.master is not None:
            out["master"] = {seg.name: self.master[seg.offset:seg.offset + seg.numel].view(seg.shape).detach().cpu().clone()
                             for seg in self.flat.segments if seg.stage == stage}
        return out

    def load_state_dict_for_stage(self, stage: int, sd: dict):
        for seg in self.flat.segments:
            if seg.stage == stage and seg.name in sd.get("momentum_buffer", {}):
                self.momentum_buffer[seg.offset:seg.offset + seg.numel].copy_(
                    sd["momentum_buffer"][seg.name].reshape(-1).to(self.momentum_buffer))
        if self.master is not None:
            for seg in self.flat.segments:
                if seg.stage != stage:
                    continue
                src = sd.get("master", {}).get(seg.name)
                dst = self.master[seg.offset:seg.offset + seg.numel]
                # without saved master weights fall back to the (rounded) model weights
                dst.copy_(src.reshape(-1) if src is not None else
                          self.flat.params[seg.offset:seg.offset + seg.numel].float())
        self.steps = max(self.steps, int(sd.get("steps", 0)))


def _weights_rewritten():
    """The step kernels rewrote parameters through raw pointers: drop weight-derived caches keyed on tensor
    versions (ops/conv.py's kernel weight layouts)."""
    from .conv import bump_weight_generation

    bump_weight_generation()
