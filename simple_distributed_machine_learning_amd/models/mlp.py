"""MNIST-shape MLPs split into pipeline stages (BASELINE configs 1-3).

* ``mlp``       784 -> 128 -> 10, 2 stages: stage 0 = fc1+ReLU, stage 1 = fc2+log_softmax
                (the north-star model; same cut position as the reference, which sends the
                flattened activation to the next rank: /root/reference/simple_distributed.py:46-49)
* ``mlp4x1024`` 784 -> 1024 x4 -> 10, 4 stages (fc1 | fc2 | fc3 | fc4+fc5)

On a ROCm device every stage runs hand-written gfx950 kernels with no autograd graph:

* hidden layer forward  : fp32 MFMA GEMM with fused bias + ReLU epilogue (large shapes: operands split
                          once into two fp16 planes, 3 MFMA products per product, ops.linear_relu_fwd_x2)
* hidden layer backward : dX GEMM with the ReLU mask fused into the A-operand load,
                          dW/db split-K MFMA GEMM accumulating straight into the flat grad buffer
* classifier head       : ONE kernel for fc2 -> log_softmax -> NLL -> backward (dlogits, dW2,
                          db2, dX) — the entire last stage of the 784-128-10 model.

On CPU the same modules run through PyTorch autograd (Gloo multi-process tests).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import ModelSpec, PipelineStage
from .. import ops


def partition_layers(n_layers: int, n_stages: int) -> List[List[int]]:
    """Contiguous layer ranges per stage; extra layers go to the LAST stages (the classifier
    head is cheap, so the last stage takes the hidden layer + head)."""
    if n_stages > n_layers:
        raise ValueError(f"cannot split {n_layers} layers into {n_stages} stages")
    base, extra = divmod(n_layers, n_stages)
    out, i = [], 0
    for s in range(n_stages):
        k = base + (1 if s >= n_stages - extra else 0)
        out.append(list(range(i, i + k)))
        i += k
    return out


class MLPStage(PipelineStage):
    """A contiguous run of Linear layers; ReLU after every layer except the final classifier."""

    def __init__(self, dims: Sequence[int], layer_ids: Sequence[int], stage_id: int, num_stages: int,
                 dropout: float = 0.0):
        super().__init__()
        self.stage_id, self.num_stages = stage_id, num_stages
        self.n_total = len(dims) - 1
        self.layer_ids = list(layer_ids)
        self.names = [f"fc{i + 1}" for i in self.layer_ids]
        for i, name in zip(self.layer_ids, self.names):
            setattr(self, name, nn.Linear(dims[i], dims[i + 1]))
        self.loss_kind = "nll"
        self.in_features = dims[self.layer_ids[0]]
        # stage 0 reads MNIST's uint8 pixels directly (ToTensor fused into fc1's GEMM)
        self.accepts_u8_pixels = self.layer_ids[0] == 0
        # fc1's bf16 weight planes, kept current by the fused SGD step (attach_plane_cache)
        self.plane_cache = None
        self.flat_ref = None

    def attach_plane_cache(self, flat, optimizer) -> bool:
        """ROCm, uint8-fed first layer: let ``optimizer``'s step write fc1's weight planes, so the
        forward skips its per-step split launch (ops.PlaneCache)."""
        if not self.accepts_u8_pixels or not flat.params.is_cuda:
            return False
        w = self.layers()[0].weight
        cache = ops.PlaneCache(w)
        if not optimizer.add_plane_cache(cache, w):
            return False
        self.plane_cache, self.flat_ref = cache, flat
        return True

    def layers(self) -> List[nn.Linear]:
        # cached: the step path asks ~10 times per step and each nn.Module attribute lookup costs ~1 us; a
        # reassigned layer attribute drops the cache (__setattr__)
        ls = self.__dict__.get("_layer_list")
        if ls is None:
            ls = self.__dict__["_layer_list"] = [getattr(self, n) for n in self.names]
        return list(ls)

    def __setattr__(self, name, value):
        if name in self.__dict__.get("names", ()):
            self.__dict__.pop("_layer_list", None)
        super().__setattr__(name, value)

    def _is_classifier(self, i: int) -> bool:
        return self.layer_ids[i] == self.n_total - 1

    def forward(self, x):
        x = ops.pixels_to_float(x.reshape(x.shape[0], -1))
        for i, lin in enumerate(self.layers()):
            x = lin(x)
            if self._is_classifier(i):
                x = F.log_softmax(x, dim=1)
            else:
                x = F.relu(x)
        return x

    # ---- fused HIP path --------------------------------------------------------------------
    def _fused(self, x) -> bool:
        return x.is_cuda

    def fwd(self, x, ctx, train, mask_out=None):
        """``mask_out`` (int32 [M, N/32], uint8-fed single-layer stage): also write the output's ReLU bits
        there (ops.relu_bits layout) - all :meth:`bwd_from_factor` needs of the output."""
        if not self._fused(x):
            if mask_out is not None:
                y = super().fwd(x, ctx, train)
                mask_out.copy_(ops.relu_bits(y))
                ctx["mask"] = mask_out
                if x.dtype == torch.uint8 and len(self.layers()) == 1 and train:
                    ctx["acts"] = [x.reshape(x.shape[0], -1)]  # bwd_from_factor's operands, as on ROCm
                return y
            return super().fwd(x, ctx, train)
        x = ops.carry_bounds(x.reshape(x.shape[0], -1), x)
        if x.dtype == torch.uint8:
            x = x.contiguous()
        elif x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        acts = [x]
        x2 = {}  # layer index -> two-fp16-plane operands kept for its backward (ops.linear_relu_fwd_x2)
        for i, lin in enumerate(self.layers()):
            assert not self._is_classifier(i), "classifier layers run in head_fwd"
            if x.dtype == torch.uint8:
                cache = self.plane_cache
                epoch = self.flat_ref.param_epoch if self.flat_ref is not None else 0
                m = mask_out if len(self.layers()) == 1 else None
                x = ops.linear_relu_fwd_u8(x, lin.weight, lin.bias, cache, epoch, mask_out=m)
                if m is not None:
                    ctx["mask"] = m
            elif ops.x2_ok(x, lin.weight):
                x, pl = ops.linear_relu_fwd_x2(x, lin.weight, lin.bias)
                if train:
                    x2[i] = pl
            else:
                x = ops.linear_relu_fwd(x, lin.weight, lin.bias)
            acts.append(x)
        if train:
            ctx["acts"] = acts
            if x2:
                ctx["x2"] = x2
        return x

    # Fused-path boundary protocol: the gradient an MLP stage sends back is already multiplied
    # by the ReLU mask of its input (= the previous stage's output), i.e. it is d/dz of the
    # previous stage's last pre-activation. The mask is applied for free where the input is
    # already in registers (head kernel, dX epilogue), and the receiving stage skips it.
    def bwd(self, grad_y, ctx):
        if "acts" not in ctx:
            return super().bwd(grad_y, ctx)
        acts = ctx.pop("acts")
        x2 = ctx.pop("x2", {})
        g = grad_y.contiguous() if not grad_y.is_contiguous() else grad_y
        layers = self.layers()
        for i in range(len(layers) - 1, -1, -1):
            lin = layers[i]
            if acts[i].dtype == torch.uint8:  # uint8 pixels: first layer, no input gradient
                ops.linear_wgrad_u8(acts[i], g, lin.weight.grad, lin.bias.grad)
                return None
            need_dx = (i > 0) or (not self.is_first)
            if i in x2:
                g = ops.linear_relu_bwd_x2(acts[i], g, lin.weight.grad, lin.bias.grad, x2.pop(i), need_dx, need_dx)
            else:
                g = ops.linear_relu_bwd(acts[i], acts[i + 1], g, lin.weight, lin.weight.grad, lin.bias.grad, need_dx,
                                        gy_masked=True, mask_dx=need_dx)
        return g

    # head_fwd(stats=..., stats_init=True) overwrites ``stats`` instead of adding to it (an engine
    # then allocates its per-step [loss, correct] without a zero-fill launch)
    supports_stats_init = True

    def head_fwd(self, x, target, ctx, train, loss_scale, stats=None, stats_init: bool = False):
        if not self._fused(x):
            loss, correct, n = super().head_fwd(x, target, ctx, train, loss_scale)
            if stats is not None:
                ops._put_stats(stats, loss.float(), correct.float(), stats_init)
                return None, None, n
            return loss, correct, n
        x = ops.carry_bounds(ops.pixels_to_float(x.reshape(x.shape[0], -1)), x)
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        layers = self.layers()
        acts = [x]
        x2 = {}
        for i in range(len(layers) - 1):
            if train and ops.x2_ok(x, layers[i].weight):
                x, x2[i] = ops.linear_relu_fwd_x2(x, layers[i].weight, layers[i].bias)
            else:
                x = ops.linear_relu_fwd(x, layers[i].weight, layers[i].bias)
            acts.append(x)
        head = layers[-1]
        need_dx = train and (len(layers) > 1 or not self.is_first)
        loss, correct, dx = ops.linear_logsoftmax_nll(
            x, head.weight, head.bias, target,
            head.weight.grad if train else None, head.bias.grad if train else None,
            loss_scale, need_dx, stats=stats, mask_dx=need_dx, stats_init=stats_init)
        if train:
            ctx["acts"] = acts
            ctx["dx"] = dx
            if x2:
                ctx["x2"] = x2
        return loss, correct, target.numel()

    # Factored boundary gradient (rotate placement): the gradient this single-Linear head sends back,
    # (dl @ W) * (x > 0), has rank <= C per sample; the head returns the factor dl [M, C] and the
    # rank that owns the boundary activation x rebuilds the gradient with ITS replica of W
    # (boundary_grad_from_factor). 40 bytes per sample cross the boundary instead of 512 for
    # 784-128-10, with a bit-identical result (ops.head_dx_from_dlogits).
    @property
    def supports_factored_grad(self) -> bool:
        return self.is_last and not self.is_first and len(self.layer_ids) == 1

    def head_fwd_factored(self, x, target, loss_scale, stats, stats_init: bool = False, defer_reduce: bool = False):
        """Training head_fwd + head_bwd in one call: returns (dl, count); loss/correct go to stats.
        ``defer_reduce``: returns (dl, count, pending) with the head's gradient/stats reduction left to
        ``pending`` (ops.linear_logsoftmax_nll_dl), which must reach :meth:`bwd_from_factor` or be run."""
        head = self.layers()[-1]
        x = x.reshape(x.shape[0], -1)
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        out = ops.linear_logsoftmax_nll_dl(x, head.weight, head.bias, target, head.weight.grad, head.bias.grad,
                                           loss_scale, stats, stats_init, defer_reduce=defer_reduce)
        if defer_reduce:
            return out[0], target.numel(), out[1]
        return out, target.numel()

    def boundary_grad_from_factor(self, dl, x):
        """d(loss)/d(pre-activation of the producing stage) from the head's factor ``dl`` and the
        boundary activation ``x`` (the producer's ReLU output)."""
        head = self.layers()[-1]
        return ops.head_dx_from_dlogits(dl, head.weight.detach(), x.reshape(x.shape[0], -1), mask=True)

    def factor_weight(self):
        """The weight the factored boundary gradient is expanded with (dx = dl @ W)."""
        return self.layers()[-1].weight.detach()

    def grad_span(self):
        """(first gradient tensor, numel) of this stage's parameters in the flat gradient buffer, if
        they are one contiguous range (their flat segments are back to back), else None."""
        ps = [p for lin in self.layers() for p in (lin.weight, lin.bias)]
        if any(p.grad is None for p in ps):
            return None
        for a, b in zip(ps, ps[1:]):
            if a.grad.data_ptr() + a.numel() * a.grad.element_size() != b.grad.data_ptr():
                return None
        return ps[0].grad, sum(p.numel() for p in ps)

    def bwd_from_factor(self, dl, w2, ctx, head_pending=None, sgd=None, groups=None, final=True) -> bool:
        """Stage-0 backward fed by the factored boundary gradient dl (dz = (dl @ w2) * (h > 0), h this
        stage's output). A single uint8-fed layer takes it straight into its weight-gradient kernel
        (dz never materialised; a deferred head reduction ``head_pending`` shares its reduction
        launch, and with ``sgd`` so does the optimizer step: ``self.sgd_fused`` tells whether it
        ran); returns False (nothing done, ``head_pending`` untouched) for other stages. ``groups``: one
        hidden-group range only (ops.linear_wgrad_u8_dl); ``final=False`` keeps ctx for the next range."""
        self.__dict__["sgd_fused"] = False  # (plain flag, bypassing nn.Module.__setattr__)
        acts = ctx.get("acts")
        layers = self.layers()
        if acts is None or len(layers) != 1 or acts[0].dtype != torch.uint8:
            return False
        mask = ctx.get("mask")  # the output's ReLU bits (fwd(mask_out=) / fwd_head_fused), else h itself
        if final:
            ctx.pop("acts")
            ctx.pop("mask", None)
        lin = layers[0]
        self.__dict__["sgd_fused"] = ops.linear_wgrad_u8_dl(acts[0], dl, w2, mask if mask is not None else acts[1],
                                                lin.weight.grad, lin.bias.grad, head_pending=head_pending, sgd=sgd,
                                                groups=groups)
        return True

    def hidden_groups(self) -> int:
        """64-unit hidden groups of a single-layer stage's output (the weight gradient's split unit)."""
        n = self.layers()[0].out_features
        return n // 64 if len(self.layers()) == 1 and n % 64 == 0 else 0

    # ---- stage 0 + stage 1 in ONE launch (both stages on this rank) -------------------------
    def can_fuse_head(self, head: "MLPStage", x: torch.Tensor) -> bool:
        """A uint8-fed single hidden layer followed by a single-Linear head (784-128-10) fuse into one
        kernel on ROCm (ops.linear_relu_head_u8): the boundary activation never reaches HBM."""
        if len(self.layers()) != 1 or self.plane_cache is None or not getattr(head, "supports_factored_grad", False):
            return False
        return ops.relu_head_u8_supported(x.reshape(x.shape[0], -1), self.layers()[0].weight, head.layers()[-1].weight)

    def fwd_head_fused(self, x, head: "MLPStage", target, loss_scale, stats, stats_init, dl_out, mask_out, ctx,
                       defer=False):
        """Training forward of this stage AND ``head``'s forward + loss + backward (its factored boundary
        gradient dl into ``dl_out``, the ReLU bits into ``mask_out``; ctx then serves
        :meth:`bwd_from_factor`). Returns (dl bounds, deferred head reduction or None)."""
        lin, hl = self.layers()[0], head.layers()[-1]
        x = x.reshape(x.shape[0], -1)
        d = self.__dict__  # (plain counter: nn.Module.__setattr__ costs ~3 us ahead of the step's first launch)
        d["fused_head_calls"] = d.get("fused_head_calls", 0) + 1
        epoch = self.flat_ref.param_epoch if self.flat_ref is not None else 0
        out = ops.linear_relu_head_u8(x, lin.weight, lin.bias, self.plane_cache, epoch, hl.weight.detach(),
                                      hl.bias.detach(), target, hl.weight.grad, hl.bias.grad, loss_scale, stats,
                                      stats_init, dl_out, mask_out, defer)
        if ctx is not None:
            ctx["acts"] = [x]
            ctx["mask"] = mask_out
        return out

    def head_bwd(self, ctx):
        if "dx" not in ctx:
            return super().head_bwd(ctx)
        acts = ctx.pop("acts")
        g = ctx.pop("dx")
        x2 = ctx.pop("x2", {})
        layers = self.layers()
        for i in range(len(layers) - 2, -1, -1):
            need_dx = (i > 0) or (not self.is_first)
            if i in x2:
                g = ops.linear_relu_bwd_x2(acts[i], g, layers[i].weight.grad, layers[i].bias.grad, x2.pop(i), need_dx,
                                           need_dx)
            else:
                g = ops.linear_relu_bwd(acts[i], acts[i + 1], g, layers[i].weight, layers[i].weight.grad,
                                        layers[i].bias.grad, need_dx, gy_masked=True, mask_dx=need_dx)
        return g


def mlp_spec(dims: Sequence[int], num_stages: int, name: str) -> ModelSpec:
    dims = list(dims)
    parts = partition_layers(len(dims) - 1, num_stages)

    def build(s: int) -> PipelineStage:
        return MLPStage(dims, parts[s], s, num_stages)

    def shape(s: int, mb: int) -> Tuple[int, ...]:
        return (mb, dims[parts[s][-1] + 1])

    return ModelSpec(name=name, num_stages=num_stages, build_stage=build, boundary_shape=shape,
                     boundary_dtype=torch.float32, input_kind="image")


MLP_DIMS = (784, 128, 10)
MLP4X1024_DIMS = (784, 1024, 1024, 1024, 1024, 10)
