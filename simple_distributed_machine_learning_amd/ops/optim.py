"""Per-stage fused SGD with momentum over the rank's flat parameter buffer.

Replaces ``DistributedOptimizer(optim.SGD, param_rrefs, lr=0.1, momentum=0.5)``
(/root/reference/simple_distributed.py:100-104, :113), which creates one TorchScript
``_FunctionalSGD`` per parameter owner and drives each step by RPC. Here each rank updates
the parameters it owns with ONE kernel launch over its flat buffer (utils/flat.py); the
update rule is torch.optim.SGD's (dampening 0, no nesterov, no weight decay by default):
``buf = momentum * buf + g`` (``buf = g`` on the first step), ``p -= lr * buf``.
"""
from __future__ import annotations

import torch

from . import sgd_momentum_
from ..utils.flat import FlatParams


class FusedSGD:
    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.flat = flat
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.momentum_buffer = torch.zeros_like(flat.params) if momentum != 0 else flat.params.new_zeros(64)
        self.steps = 0

    def step(self, zero_grad: bool = True):
        """One update. ``zero_grad`` clears the gradients inside the same kernel (the engine
        then skips its own zero_grad at the next step: one launch, one pass over memory)."""
        sgd_momentum_(self.flat.params, self.flat.grads, self.momentum_buffer, self.lr, self.momentum,
                      self.dampening, self.weight_decay, self.nesterov, self.steps == 0, zero_grad)
        if zero_grad:
            self.flat.grads_zero = True
        self.steps += 1

    def zero_grad(self):
        self.flat.zero_grad()

    # ---- checkpoint (per-parameter names, reference-compatible keys) ----------------------
    def state_dict_for_stage(self, stage: int) -> dict:
        bufs = {}
        for seg in self.flat.segments:
            if seg.stage == stage and self.momentum != 0:
                bufs[seg.name] = self.momentum_buffer[seg.offset:seg.offset + seg.numel].view(seg.shape).detach().cpu().clone()
        return {"momentum_buffer": bufs, "steps": self.steps, "lr": self.lr, "momentum": self.momentum,
                "dampening": self.dampening, "weight_decay": self.weight_decay, "nesterov": self.nesterov}

    def load_state_dict_for_stage(self, stage: int, sd: dict):
        for seg in self.flat.segments:
            if seg.stage == stage and seg.name in sd.get("momentum_buffer", {}):
                self.momentum_buffer[seg.offset:seg.offset + seg.numel].copy_(
                    sd["momentum_buffer"][seg.name].reshape(-1).to(self.momentum_buffer))
        self.steps = max(self.steps, int(sd.get("steps", 0)))
