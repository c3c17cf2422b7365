"""Linear layer whose backward writes weight/bias gradients straight into ``param.grad``.

In the pipeline engine every parameter's ``.grad`` is a view into the rank's flat gradient
buffer (utils/flat.py), and each micro-batch ADDS its gradient there. Stock autograd first
materialises each gradient and then launches an AccumulateGrad add (``grad += new``), so
every weight and bias costs an extra full read and write per micro-batch. It also reduces
the bias gradient with a generic reduction. This module avoids both:

* dW (bf16 on ROCm): ``wgrad_bf16_``, a hand-written MFMA GEMM (csrc/kernels/gemm_bf16_wgrad.hip)
  that splits the token reduction over workgroups and adds the result into the bf16 gradient
  in place. hipBLASLt runs these small-output / long-reduction shapes at 180-470 TF/s
  (tools/bench_gpt2_gemms.py). Other dtypes: ``param.grad.addmm_(gy^T, x)`` (beta = 1).
* db (bf16 on ROCm): fused into ``wgrad_bf16_`` (the weight-gradient GEMM already stages every
  gy tile; its first column tile sums them); otherwise ``bias_grad_bf16_``, a deterministic
  two-pass column sum that adds into the bf16 gradient in place (csrc/kernels/transformer.hip).

When a parameter has no ``.grad`` yet (standalone use), the gradients are returned to
autograd in the usual way. CPU tensors and non-bf16 dtypes keep the plain ``F.linear``
path. The GEMMs themselves are plain library GEMMs (hipBLASLt) for the forward and input gradient.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import kernels


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.addmm(b, x2, w.t()) if b is not None else x2 @ w.t()
        ctx.save_for_backward(x2)
        ctx.w, ctx.b = w, b  # the Parameters themselves: their .grad is written in backward
        ctx.in_shape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        (x2,) = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        g2 = gy.reshape(-1, gy.shape[-1])
        dx = (g2 @ w).view(ctx.in_shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        bias_done = False
        if ctx.needs_input_grad[1]:
            if w.grad is not None and _wgrad_ok(g2, x2, w.grad):
                fuse_b = (b is not None and ctx.needs_input_grad[2] and b.grad is not None
                          and b.grad.is_contiguous() and b.grad.dtype == torch.bfloat16)
                kernels().wgrad_bf16_(g2, x2, w.grad, b.grad if fuse_b else None)
                bias_done = fuse_b
            elif w.grad is not None:
                w.grad.addmm_(g2.t(), x2)
            else:
                gw = g2.t() @ x2
        if b is not None and ctx.needs_input_grad[2] and not bias_done:
            if b.grad is not None and b.grad.is_contiguous() and g2.stride(-1) == 1:
                kernels().bias_grad_bf16_(g2, b.grad)
            else:
                gb = g2.sum(0)
        return dx, gw, gb


def _wgrad_ok(g2, x2, gw) -> bool:
    return (g2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and gw.dtype == torch.bfloat16
            and g2.stride(-1) == 1 and x2.stride(-1) == 1 and gw.is_contiguous()
            and g2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0
            and kernels().wgrad_bf16_supported(gw.shape[0], gw.shape[1], g2.shape[0]))


def linear(x, w, b=None):
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        return _LinearFn.apply(x, w, b)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """nn.Linear (same parameter names and init) with the fused-gradient backward on ROCm bf16."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
