"""Autograd wrappers of the transformer kernels (csrc/kernels/transformer.hip).

On ROCm bf16 tensors they run the hand-written gfx950 kernels; anything else falls back
to the plain PyTorch definition (CPU tests, fp32 tiny models).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import kernels


def _hip_bf16(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        xc = x.contiguous()
        y, mean, rstd = kernels().layernorm_fwd_bf16(xc, w, b, eps)
        ctx.save_for_backward(xc, w, mean, rstd)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, mean, rstd = ctx.saved_tensors
        wp, bp = ctx.params
        if wp.grad is not None and bp.grad is not None and wp.grad.is_contiguous() and bp.grad.is_contiguous():
            # flat-buffer gradients: dw/db are added in place by the reduction kernel
            dx = kernels().layernorm_bwd_bf16_accum(x, w, gy.contiguous(), mean, rstd, wp.grad, bp.grad)
            return dx, None, None, None
        dx, dw, db = kernels().layernorm_bwd_bf16(x, w, gy.contiguous(), mean, rstd)
        return dx, dw.to(w.dtype), db.to(w.dtype), None


def layer_norm(x, w, b, eps: float = 1e-5):
    if _hip_bf16(x, w, b) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 4096:
        return _LayerNormFn.apply(x, w, b, eps)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


class _LayerNormPassFn(torch.autograd.Function):
    """(x, LayerNorm(x)) for an x that also feeds a residual path: the backward adds the residual-path gradient inside
    the LayerNorm backward kernel (fp32, rounded once) instead of autograd summing the two bf16 gradients with a
    separate add kernel (GPT-2: each stage's first block)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        xc = x.contiguous()
        y, mean, rstd = kernels().layernorm_fwd_bf16(xc, w, b, eps)
        ctx.save_for_backward(xc, w, mean, rstd)
        ctx.params = (w, b)
        return xc.view_as(xc), y

    @staticmethod
    def backward(ctx, g_x, g_y):
        x, w, mean, rstd = ctx.saved_tensors
        wp, bp = ctx.params
        g_x = None if g_x is None else g_x.contiguous()
        if g_y is None:
            return g_x, None, None, None
        if wp.grad is not None and bp.grad is not None and wp.grad.is_contiguous() and bp.grad.is_contiguous():
            d = kernels().layernorm_bwd_bf16_accum(x, w, g_y.contiguous(), mean, rstd, wp.grad, bp.grad, g_x)
            return d, None, None, None
        d, dw, db = kernels().layernorm_bwd_bf16(x, w, g_y.contiguous(), mean, rstd)
        if g_x is not None:
            d = d + g_x
        return d, dw.to(w.dtype), db.to(w.dtype), None


def layer_norm_pass(x, ln: nn.LayerNorm):
    """(x, ln(x)), both differentiable; on ROCm bf16 the two gradients of x meet inside the LayerNorm backward."""
    w, b = ln.weight, ln.bias
    if _hip_bf16(x, w, b) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 4096:
        return _LayerNormPassFn.apply(x, w, b, ln.eps)
    return x, ln(x)


class _AddLayerNormFn(torch.autograd.Function):
    """xs = x + h; y = LayerNorm(xs) in one pass. Backward: dxs = g_xs + LN_bwd(g_y), added inside
    the LayerNorm backward kernel; both addends of the residual get dxs."""

    @staticmethod
    def forward(ctx, x, h, w, b, eps):
        xs, y, mean, rstd = kernels().add_layernorm_fwd_bf16(x.contiguous(), h.contiguous(), w, b, eps)
        ctx.save_for_backward(xs, w, mean, rstd)
        ctx.params = (w, b)
        return xs, y

    @staticmethod
    def backward(ctx, g_xs, g_y):
        xs, w, mean, rstd = ctx.saved_tensors
        wp, bp = ctx.params
        g_xs = None if g_xs is None else g_xs.contiguous()
        if wp.grad is not None and bp.grad is not None and wp.grad.is_contiguous() and bp.grad.is_contiguous():
            d = kernels().layernorm_bwd_bf16_accum(xs, w, g_y.contiguous(), mean, rstd, wp.grad, bp.grad, g_xs)
            return d, d, None, None, None
        d, dw, db = kernels().layernorm_bwd_bf16(xs, w, g_y.contiguous(), mean, rstd)
        if g_xs is not None:
            d = d + g_xs
        return d, d, dw.to(w.dtype), db.to(w.dtype), None


def add_layer_norm(x, h, ln: nn.LayerNorm):
    """(x + h, ln(x + h)): the residual add fused into the LayerNorm pass on ROCm bf16."""
    w, b = ln.weight, ln.bias
    if _hip_bf16(x, h, w, b) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 4096 and x.shape == h.shape:
        return _AddLayerNormFn.apply(x, h, w, b, ln.eps)
    xs = x + h
    return xs, ln(xs)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameter names) backed by the HIP kernel for bf16 on ROCm."""

    def forward(self, x):
        return layer_norm(x, self.weight, self.bias, self.eps)


def cross_entropy_sum(logits, target, scale: float, need_grad: bool, ignore_index: int = -100):
    """Summed token cross-entropy on [rows, V] logits.

    Returns (loss_sum, correct, count, dlogits): dlogits = scale * d(loss_sum)/dlogits in the
    logits dtype (None unless ``need_grad``). bf16 on ROCm uses the fused single-row kernel
    (never materialises fp32 logits)."""
    if _hip_bf16(logits):
        if not (logits.stride(-1) == 1 and (logits.shape[0] <= 1 or logits.stride(0) >= logits.shape[1])):
            logits = logits.contiguous()  # (rows may be padded: the lm_head's [T, 50304]-strided logits stay in place)
        loss, ok, g = kernels().cross_entropy_bf16(logits, target.contiguous(), float(scale),
                                                   ignore_index, need_grad)
        valid = int((target != ignore_index).sum()) if ignore_index >= 0 else target.numel()
        return loss.sum(), ok.sum(), valid, g
    z = logits.float().detach().requires_grad_(need_grad)
    with torch.enable_grad():
        loss = F.cross_entropy(z, target, reduction="sum", ignore_index=ignore_index)
    g = None
    if need_grad:
        (g,) = torch.autograd.grad(loss * scale, z)
        g = g.to(logits.dtype)
    valid = target != ignore_index
    correct = ((z.detach().argmax(1) == target) & valid).sum()
    # no host sync unless an ignore_index can actually occur (keeps the step graph-capturable)
    count = target.numel() if ignore_index < 0 else int(valid.sum())
    return loss.detach(), correct, count, g


class _FlashAttnFn(torch.autograd.Function):
    """Causal attention on a fused qkv projection [B, S, 3C] (HIP kernels, bf16, d = 64)."""

    @staticmethod
    def forward(ctx, qkv, n_head: int, scale: float):
        B, S, C3 = qkv.shape
        C = C3 // 3
        D = C // n_head
        qkv = qkv.contiguous()
        q, k, v = (qkv[..., i * C:(i + 1) * C].view(B, S, n_head, D) for i in range(3))
        out, lse = kernels().attention_fwd(q, k, v, scale, True)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_head, ctx.scale = n_head, scale
        return out.view(B, S, C)

    @staticmethod
    def backward(ctx, gout):
        qkv, out, lse = ctx.saved_tensors
        B, S, C3 = qkv.shape
        C, H = C3 // 3, ctx.n_head
        D = C // H
        dqkv = torch.empty_like(qkv)
        q, k, v = (qkv[..., i * C:(i + 1) * C].view(B, S, H, D) for i in range(3))
        dq, dk, dv = (dqkv[..., i * C:(i + 1) * C].view(B, S, H, D) for i in range(3))
        kernels().attention_bwd(q, k, v, out, gout.contiguous().view(B, S, H, D), lse, dq, dk, dv, ctx.scale, True)
        return dqkv, None, None


def causal_attention(qkv, n_head: int):
    """softmax(q k^T / sqrt(d), causal) v from a fused [B, S, 3C] projection -> [B, S, C]."""
    B, S, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    if _hip_bf16(qkv) and D == 64:
        return _FlashAttnFn.apply(qkv, n_head, 1.0 / math.sqrt(D))
    q, k, v = qkv.split(C, dim=2)
    q = q.view(B, S, n_head, D).transpose(1, 2)
    k = k.view(B, S, n_head, D).transpose(1, 2)
    v = v.view(B, S, n_head, D).transpose(1, 2)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    return y.transpose(1, 2).contiguous().view(B, S, C)


class _GeluFn(torch.autograd.Function):
    """tanh-GELU on the HIP kernels (gpt2_ops.hip); the backward multiplies in place."""

    @staticmethod
    def forward(ctx, x):
        xc = x.contiguous()
        ctx.save_for_backward(xc)
        return kernels().gelu_fwd_bf16(xc)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return kernels().gelu_bwd_bf16(gy.contiguous(), x, False)


def gelu(x):
    """GELU with the tanh approximation (GPT-2's activation)."""
    if _hip_bf16(x) and x.numel() % 8 == 0:
        return _GeluFn.apply(x)
    return F.gelu(x, approximate="tanh")


class _EmbeddingFn(torch.autograd.Function):
    """wte[tok] + wpe[:S] (HIP gather). The backward adds into wte.grad / wpe.grad in place (flat
    gradient buffer) with a deterministic segmented sum over the stably sorted tokens."""

    @staticmethod
    def forward(ctx, tok, wte, wpe):
        tok = tok.contiguous()
        out = kernels().embedding_fwd_bf16(tok, wte, wpe)
        ctx.tok = tok
        ctx.params = (wte, wpe)
        return out

    @staticmethod
    def backward(ctx, g):
        wte, wpe = ctx.params
        g = g.contiguous()
        sorted_tok, perm = torch.sort(ctx.tok.reshape(-1), stable=True)
        direct = all(p.grad is not None and p.grad.is_contiguous() and p.grad.dtype == torch.bfloat16
                     for p in (wte, wpe))
        if direct:
            kernels().embedding_bwd_bf16(g, sorted_tok, perm, wte.grad, wpe.grad)
            return None, None, None
        gwte, gwpe = torch.zeros_like(wte), torch.zeros_like(wpe)
        kernels().embedding_bwd_bf16(g, sorted_tok, perm, gwte, gwpe)
        return None, gwte, gwpe


def embedding(tok, wte, wpe):
    """GPT-2 input embedding: wte[tok] + wpe[position] for tok [B, S]."""
    if _hip_bf16(wte, wpe) and tok.is_cuda and wte.shape[1] % 4 == 0:
        return _EmbeddingFn.apply(tok, wte, wpe)
    S = tok.shape[1]
    return F.embedding(tok, wte) + F.embedding(torch.arange(S, device=tok.device), wpe)[None]
