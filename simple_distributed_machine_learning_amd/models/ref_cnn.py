"""The reference's own model: the PyTorch-examples MNIST CNN split after the conv stack.

Stage 0 (reference ``Network1``, /root/reference/simple_distributed.py:26-50):
    conv1(1->10,k5) -> maxpool2 -> relu -> conv2(10->20,k5) -> Dropout2d(0.5) -> maxpool2
    -> relu -> flatten(320)
Stage 1 (reference ``Network2``, :60-80):
    fc1(320->50) -> relu -> dropout(0.5) -> fc2(50->10) -> log_softmax

``state_dict`` keys match the reference exactly (stage 0: conv1.*, conv2.*; stage 1:
fc1.*, fc2.*), so per-stage checkpoints are interchangeable.

Reference quirk (Appendix B.3): ``F.dropout`` in Network2 has no ``training=`` argument, so
it stays active during ``test()``. ``eval_dropout=True`` (default) reproduces that;
``False`` gives the conventional behaviour.

On ROCm devices each stage pass is ONE fused HIP launch (csrc/kernels/ref_cnn.hip): stage 0
forward, stage 0 backward (recompute), and stage 1 forward+NLL+backward. At the reference's
batch of 60 the model is launch-bound, so fusing ~30 PyTorch/MIOpen launches per step into 3
is the whole game. Dropout masks there come from a counter hash keyed by a per-pass seed drawn
from torch's CPU generator (so ``torch.manual_seed`` and the checkpointed RNG state still
determine them); CPU tensors keep PyTorch's own dropout. The stage boundary tensor
[mb, 320] moves over RCCL exactly like the MLP's.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import ModelSpec, PipelineStage
from .. import ops


def _draw_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _RngStage(PipelineStage):
    """Stage whose fused kernels draw dropout masks; ``rng_step`` is an int64 device counter
    (the engine attaches its own; a non-persistent buffer keeps the reference's state_dict
    keys)."""
    uses_rng_step = True

    def _ctr(self, x):
        ctr = getattr(self, "rng_step", None)
        return ctr if ctr is not None and ctr.device == x.device else None


class Network1Stage(_RngStage):
    def __init__(self, dropout: float = 0.5):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d(p=dropout)
        self.loss_kind = "nll"

    def forward(self, x):
        z1 = F.relu(F.max_pool2d(self.conv1(x), 2))
        z2 = self.conv2(z1)
        z3 = F.relu(F.max_pool2d(self.conv2_drop(z2), 2))
        return z3.reshape(-1, 320)

    # ---- fused HIP path (one launch each way) ---------------------------------------------
    def fwd(self, x, ctx, train):
        if not x.is_cuda:
            return super().fwd(x, ctx, train)
        x = x.float().contiguous()
        p = self.conv2_drop.p
        drop = train and p > 0
        seed = _draw_seed() if drop else 0
        ctr = self._ctr(x)
        y, saved = ops.ref_cnn_stage0_fwd(x, self.conv1, self.conv2, seed, p, drop, ctr=ctr, save=train)
        if train:
            ctx.update(x=x, y=y, saved=saved, seed=seed, drop=drop, ctr=ctr)
        return y

    def bwd(self, grad_y, ctx):
        if "seed" not in ctx:
            return super().bwd(grad_y, ctx)
        ops.ref_cnn_stage0_bwd(ctx.pop("x"), self.conv1, self.conv2, ctx.pop("y"), grad_y, ctx.pop("saved"),
                               ctx.pop("seed"), self.conv2_drop.p, ctx.pop("drop"), ctr=ctx.pop("ctr"))
        return None


class Network2Stage(_RngStage):
    def __init__(self, eval_dropout: bool = True, dropout: float = 0.5):
        super().__init__()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 10)
        self.eval_dropout = eval_dropout
        self.p = dropout
        self.loss_kind = "nll"

    def forward(self, x):
        z4 = F.dropout(F.relu(self.fc1(x)), p=self.p, training=self.training or self.eval_dropout)
        z5 = self.fc2(z4)
        return F.log_softmax(z5, dim=1)

    # ---- fused HIP path: forward + NLL + full backward in one launch ------------------------
    def head_fwd(self, x, target, ctx, train, loss_scale, stats=None):
        if not x.is_cuda:
            return super().head_fwd(x, target, ctx, train, loss_scale)
        x = x.float().contiguous()
        drop = (train or self.eval_dropout) and self.p > 0
        seed = _draw_seed() if drop else 0
        st = stats if stats is not None else torch.zeros(2, device=x.device)
        dx = ops.ref_cnn_stage1(x, self.fc1, self.fc2, target, seed, self.p, drop, loss_scale, st, train,
                                ctr=self._ctr(x))
        if train:
            ctx["dx"] = dx
        if stats is not None:
            return None, None, target.numel()
        return st[0], st[1], target.numel()

    def head_bwd(self, ctx):
        if "dx" not in ctx:
            return super().head_bwd(ctx)
        return ctx.pop("dx")


class RefCNNSingle(nn.Module):
    """Both stages in one module (single-process parity reference)."""

    def __init__(self, s0: Network1Stage, s1: Network2Stage):
        super().__init__()
        self.s0, self.s1 = s0, s1

    def forward(self, x):
        return self.s1(self.s0(x))


def ref_cnn_spec(num_stages: int = 2, eval_dropout: bool = True, dropout: float = 0.5) -> ModelSpec:
    """``dropout`` = 0.5 is the reference; 0 makes the model deterministic (parity tests)."""
    if num_stages != 2:
        raise ValueError("ref_cnn is defined as the reference's 2-stage split")

    def build(s: int) -> PipelineStage:
        return Network1Stage(dropout) if s == 0 else Network2Stage(eval_dropout, dropout)

    def shape(s: int, mb: int):
        return (mb, 320)

    return ModelSpec(name="ref_cnn", num_stages=2, build_stage=build, boundary_shape=shape,
                     boundary_dtype=torch.float32, input_kind="image")
