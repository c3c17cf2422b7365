"""Pipeline-stage protocol.

A model is a list of :class:`PipelineStage` modules cut at layer boundaries (the reference
cuts its CNN after ``view(-1, 320)``: /root/reference/simple_distributed.py:46-49). The
engine drives each stage with four hooks instead of distributed autograd
(:109-112 there):

* ``fwd(x, ctx, train)``               -> boundary output (detached), stash in ``ctx``
* ``bwd(grad_y, ctx)``                 -> grad wrt the stage input (None for stage 0)
* last stage: ``head_fwd(x, target, ctx, train, loss_scale)`` -> (loss_sum, correct, count)
* last stage: ``head_bwd(ctx)``        -> grad wrt the stage input

Default implementations use PyTorch autograd on the stage's own graph (works for any
``nn.Module``). Stages with hand-fused HIP paths (models/mlp.py) override them with explicit
kernels that never build an autograd graph.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class PipelineStage(nn.Module):
    stage_id: int = 0
    num_stages: int = 1
    # "nll": stage output is log-probabilities (reference: log_softmax + nll_loss, :79, :111)
    # "ce": stage output is logits (cross-entropy)
    loss_kind: str = "nll"
    # True if stage 0 takes uint8 pixel batches itself (ToTensor's /255 fused into its first
    # kernel); otherwise the engine converts them with ops.pixels_to_float first
    accepts_u8_pixels: bool = False

    @property
    def is_first(self) -> bool:
        return self.stage_id == 0

    @property
    def is_last(self) -> bool:
        return self.stage_id == self.num_stages - 1

    # ---- generic autograd implementation -------------------------------------------------
    def fwd(self, x: torch.Tensor, ctx: dict, train: bool) -> torch.Tensor:
        if not train:
            with torch.no_grad():
                return self(x)
        if not self.is_first:
            x = x.detach().requires_grad_(True)
        with torch.enable_grad():
            y = self(x)
        ctx["x"] = x
        ctx["y"] = y
        return y.detach()

    def bwd(self, grad_y: torch.Tensor, ctx: dict) -> Optional[torch.Tensor]:
        y = ctx.pop("y")
        x = ctx.pop("x")
        torch.autograd.backward(y, grad_y)
        return None if self.is_first else x.grad

    def loss_terms(self, out: torch.Tensor, target: torch.Tensor):
        """(loss_sum, correct, count) for one micro-batch."""
        if out.dim() > 2:  # token models: [B, S, V]
            out = out.reshape(-1, out.shape[-1])
            target = target.reshape(-1)
        if self.loss_kind == "nll":
            loss = F.nll_loss(out, target, reduction="sum")
        else:
            loss = F.cross_entropy(out.float(), target, reduction="sum")
        correct = (out.argmax(dim=1) == target).sum()
        return loss, correct, target.numel()

    def head_fwd(self, x: torch.Tensor, target: torch.Tensor, ctx: dict, train: bool, loss_scale: float,
                 stats: Optional[torch.Tensor] = None):
        """Returns (loss_sum, correct, count); a stage may instead accumulate loss/correct into
        ``stats`` in-kernel and return (None, None, count)."""
        if not train:
            with torch.no_grad():
                out = self(x)
                loss, correct, n = self.loss_terms(out, target)
            return loss.detach(), correct, n
        if not self.is_first:
            x = x.detach().requires_grad_(True)
        with torch.enable_grad():
            out = self(x)
            loss, correct, n = self.loss_terms(out, target)
        ctx["x"] = x
        ctx["loss"] = loss * loss_scale
        return loss.detach(), correct.detach(), n

    def head_bwd(self, ctx: dict) -> Optional[torch.Tensor]:
        loss = ctx.pop("loss")
        x = ctx.pop("x")
        loss.backward()
        return None if self.is_first else x.grad


@dataclass
class ModelSpec:
    """Everything the engine needs to know about a split model."""
    name: str
    num_stages: int
    build_stage: Callable[[int], PipelineStage]          # stage id -> module (CPU, fp32/dtype)
    boundary_shape: Callable[[int, int], Tuple[int, ...]]  # (stage producing, mb size) -> shape
    boundary_dtype: torch.dtype = torch.float32
    input_kind: str = "image"   # image | tokens
    param_dtype: torch.dtype = torch.float32
    vocab_size: int = 0         # token models: vocabulary size
    num_classes: int = 10       # image models: classifier outputs (label range checked under debug_sync)
    seq_len: int = 0            # token models: sequence length of the boundary tensors


def stage_seed(base_seed: int, stage: int) -> int:
    """Deterministic per-stage init seed: replicas of a stage on different ranks start equal."""
    return (base_seed * 1000003 + 7919 * (stage + 1)) % (2 ** 31 - 1)


def build_stages(spec: ModelSpec, stage_ids: Sequence[int], base_seed: int = 0) -> List[PipelineStage]:
    mods = []
    for s in stage_ids:
        torch.manual_seed(stage_seed(base_seed, s))
        m = spec.build_stage(s)
        m.stage_id = s
        m.num_stages = spec.num_stages
        mods.append(m)
    return mods
