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
path. The forward / input-gradient GEMMs run on gemm_bf16.hip's NT kernel (SDML_GPT2_GEMM=hand, the default since
its 256 x 192 tiles; SDML_GPT2_GEMM=lib puts them on hipBLASLt); the MLP's c_fc forward and c_proj input gradient
carry the GELU in their epilogues (:func:`mlp_gelu`). GPT-2's 50257-wide lm_head runs padded to 50304 rows in place
(:func:`lm_head`), so no GEMM of the GPT-2 step is left on the library.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import kernels
from . import side_stream
from .side_stream import join_side_streams  # noqa: F401 (re-export for the engine)


# SDML_GPT2_GEMM=hand (default): the forward and input-gradient GEMMs of these Linears on gemm_bf16.hip's 4-phase NT
# kernel (256 x 256 or 256 x 192 tiles, whichever fills the 256 CUs' rounds better) instead of hipBLASLt; the input
# gradient dY W runs as NT against W^T, derived once per weight per optimizer step (keyed like the conv layouts:
# ops/conv.py WEIGHT_GEN). Round 5, GPT-2 step at 16 x 1024 tokens on one MI355X: 21.69 / 21.67 ms hand vs 21.83 /
# 21.75 ms on hipBLASLt with its tuned solution table (profiles/r5_gpt2_hand_vs_lib.jsonl). "lib": hipBLASLt.
_HAND = os.environ.get("SDML_GPT2_GEMM", "hand") == "hand"
_WT = {}
EPI_STORE, EPI_BIAS = 0, 1  # csrc/kernels/kernels.h GemmEpi


def _hand_ok(x2, w) -> bool:
    if not (_HAND and x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x2.stride(-1) == 1
            and w.is_contiguous()):
        return False
    k = kernels()
    M, Kd, N = x2.shape[0], x2.shape[1], w.shape[0]
    return bool(k.gemm_bf16_supported(M, N, Kd, x2.stride(0), Kd, False)
                and k.gemm_bf16_supported(M, Kd, N, N, N, False))


# Every weight whose W^T the hand GEMMs asked for keeps one transposed buffer across optimizer steps (_WT_KNOWN: id ->
# (weakref, buffer)). The first W^T request after an optimizer step re-derives it for ALL live known weights in one
# launch (transpose_batched_bf16): per weight it was one copy launch of ~5 us, 48 per GPT-2 step. Reusing the buffers is
# safe as for the conv layouts (ops/conv.py _KNOWN): a step's backward reads them before the optimizer step that bumps
# WEIGHT_GEN, and the next step's backward re-derives them after it.
_WT_KNOWN = {}
_WT_BATCH = os.environ.get("SDML_WT_BATCH", "1") != "0"  # (A/B: 0 = one transpose copy per weight)


def _w_t(w):
    """w^T, contiguous, cached for the optimizer step (not while a hipGraph is being captured)."""
    from .conv import WEIGHT_GEN, _cache_get, _cache_put

    if torch.cuda.is_current_stream_capturing():
        return w.t().contiguous()
    key = (w.data_ptr(), w._version, WEIGHT_GEN[0], tuple(w.shape))
    hit = _cache_get(_WT, w)
    if hit is not None and hit[0] == key:
        return hit[1]
    if not (_WT_BATCH and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous()
            and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0):
        wt = w.t().contiguous()
        _cache_put(_WT, w, (key, wt))
        return wt
    import weakref

    kn = _WT_KNOWN.get(id(w))
    if kn is None or kn[0]() is not w:
        k = id(w)

        def _gone(r, k=k):
            if _WT_KNOWN.get(k, (None,))[0] is r:
                _WT_KNOWN.pop(k, None)

        _WT_KNOWN[k] = (weakref.ref(w, _gone), torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device))
    todo = []  # this weight and every other live known one whose W^T is stale
    for ref, buf in list(_WT_KNOWN.values()):
        ww = ref()
        if (ww is None or ww.device != w.device or ww.dtype != torch.bfloat16 or not ww.is_contiguous()
                or tuple(buf.shape) != tuple(ww.shape[::-1])):
            continue
        kk = (ww.data_ptr(), ww._version, WEIGHT_GEN[0], tuple(ww.shape))
        h = _cache_get(_WT, ww)
        if h is not None and h[0] == kk:
            continue
        todo.append((ww, buf, kk))
    kernels().transpose_batched_bf16([t[0] for t in todo], [t[1] for t in todo])
    for ww, buf, kk in todo:
        _cache_put(_WT, ww, (kk, buf))
    hit = _cache_get(_WT, w)
    if hit is None or hit[0] != key:  # the requesting weight itself was filtered out (e.g. resized in place)
        wt = w.t().contiguous()
        _cache_put(_WT, w, (key, wt))
        return wt
    return hit[1]


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.hand = _hand_ok(x2, w)
        if ctx.hand:
            y, _ = kernels().gemm_bf16(x2, w, b, False, EPI_BIAS if b is not None else EPI_STORE)
        else:
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
        wt = _w_t(w) if (ctx.needs_input_grad[0] and ctx.hand and g2.stride(-1) == 1) else None
        # the weight gradient first when it goes to the side stream (it then runs beside the input gradient); with
        # SDML_LINEAR_WGRAD_AFTER=1 it is enqueued after the input gradient, waiting on an event recorded before it
        side = _on_side(g2)
        ready = side_stream.ready_event(g2) if side and _WGRAD_AFTER else None
        if side and ready is None:
            gw, gb = _param_grads(g2, x2, w, b, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        dx = None
        if ctx.needs_input_grad[0]:
            if wt is not None:
                dx, _ = kernels().gemm_bf16(g2, wt, None, False, EPI_STORE)
                dx = dx.view(ctx.in_shape)
            else:
                dx = (g2 @ w).view(ctx.in_shape)
        if not side or ready is not None:
            gw, gb = _param_grads(g2, x2, w, b, ctx.needs_input_grad[1], ctx.needs_input_grad[2], ready)
        return dx, gw, gb


# weight gradients on a side stream beside the input gradient (ops/side_stream.py)
_WGRAD_AFTER = os.environ.get("SDML_LINEAR_WGRAD_AFTER", "0") == "1"


def _on_side(g2):
    return side_stream.on_side(g2)


def _wgrad_launch(g2, x2, gw, gb, ready=None):
    """gw (+ gb) += the weight (bias) gradient, on the side stream when it is on (ops/side_stream.py)."""
    side_stream.launch(lambda: kernels().wgrad_bf16_(g2, x2, gw, gb), g2, x2, ready=ready)


def _param_grads(g2, x2, w, b, need_w: bool, need_b: bool, ready=None):
    """Weight / bias gradients of y = x w^T + b from g2 = dy: added in place into the flat-buffer .grad
    (returns None for those) or returned for autograd to accumulate."""
    gw = gb = None
    bias_done = False
    if need_w:
        if w.grad is not None and _wgrad_ok(g2, x2, w.grad):
            fuse_b = (b is not None and need_b and b.grad is not None
                      and b.grad.is_contiguous() and b.grad.dtype == torch.bfloat16)
            _wgrad_launch(g2, x2, w.grad, b.grad if fuse_b else None, ready)
            bias_done = fuse_b
        elif w.grad is not None:
            w.grad.addmm_(g2.t(), x2)
        else:
            gw = g2.t() @ x2
    if b is not None and need_b and not bias_done:
        if b.grad is not None and b.grad.is_contiguous() and g2.stride(-1) == 1:
            kernels().bias_grad_bf16_(g2, b.grad)
        else:
            gb = g2.sum(0)
    return gw, gb


EPI_BIAS_GELU, EPI_DGELU = 5, 6  # csrc/kernels/kernels.h GemmEpi
EPI_BIAS_GELU_SAVE_GRAD, EPI_MUL_GRAD = 7, 8
# SDML_GELU_SAVE=grad (default): the c_fc forward saves bf16(gelu'(U)) instead of U, so the c_proj input-gradient
# epilogue is one multiply (its tanh moves into the forward epilogue, which already evaluates the sigmoid);
# "u" keeps U and evaluates gelu'(U) in the backward (exactly the unfused GELU kernels' bits)
_GELU_EPI = ((EPI_BIAS_GELU_SAVE_GRAD, EPI_MUL_GRAD) if os.environ.get("SDML_GELU_SAVE", "grad") == "grad"
             else (EPI_BIAS_GELU, EPI_DGELU))


class _MLPFn(torch.autograd.Function):
    """GPT-2's MLP, y = c_proj(gelu(c_fc(x))), with the activation fused into the GEMMs on both sides
    (gemm_bf16.hip): the c_fc forward writes gelu(U) and gelu'(U) from its epilogue, and the c_proj input-gradient
    GEMM multiplies by gelu'(U) in its epilogue - no standalone GELU passes over the [tokens, 3072] activations.
    The other two GEMMs (c_proj forward, c_fc input gradient) run on the same hand NT kernel (SDML_GPT2_GEMM=hand,
    the default; "lib" puts them on hipBLASLt); weight gradients as Linear.

    Numerics: the default save mode (SDML_GELU_SAVE=grad) rounds gelu'(U) to bf16 in the forward epilogue before the
    backward multiplies by it, so results are not bit-identical to an unfused GELU pair; SDML_GELU_SAVE=u keeps U and
    evaluates gelu'(U) in fp32 in the backward epilogue (the exact mode). GPT-2 is not in the reference, so parity is
    pinned only by the composed-kernel test (tests/test_gpt2_ops_gpu.py)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x2 = x.reshape(-1, x.shape[-1])
        a, u = kernels().gemm_bf16(x2, w1, b1, False, _GELU_EPI[0])
        y = kernels().gemm_bf16(a, w2, b2, False, EPI_BIAS)[0] if _HAND else torch.addmm(b2, a, w2.t())
        ctx.save_for_backward(x2, u, a)
        ctx.params = (w1, b1, w2, b2)
        ctx.in_shape = x.shape
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, u, a = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        g2 = gy.reshape(-1, gy.shape[-1])
        if _HAND and g2.stride(-1) == 1:  # NT against W2^T (the 256 x 128 two-workgroups-per-CU kernel)
            du, _ = kernels().gemm_bf16(g2, _w_t(w2), None, False, _GELU_EPI[1], u)
        else:
            du, _ = kernels().gemm_bf16(g2, w2, None, True, _GELU_EPI[1], u)  # (dY W2) * gelu'(U)
        gw2, gb2 = _param_grads(g2, a, w2, b2, ctx.needs_input_grad[3], ctx.needs_input_grad[4])
        w1t = _w_t(w1) if (ctx.needs_input_grad[0] and _HAND and du.stride(-1) == 1) else None
        side = _on_side(du)
        ready = side_stream.ready_event(du) if side and _WGRAD_AFTER else None
        if side and ready is None:  # (as in _LinearFn: the side-stream weight gradient first)
            gw1, gb1 = _param_grads(du, x2, w1, b1, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        dx = None
        if ctx.needs_input_grad[0]:
            if w1t is not None:
                dx, _ = kernels().gemm_bf16(du, w1t, None, False, EPI_STORE)
                dx = dx.view(ctx.in_shape)
            else:
                dx = (du @ w1).view(ctx.in_shape)
        if not side or ready is not None:
            gw1, gb1 = _param_grads(du, x2, w1, b1, ctx.needs_input_grad[1], ctx.needs_input_grad[2], ready)
        return dx, gw1, gb1, gw2, gb2


def mlp_gelu(x, w1, b1, w2, b2):
    """c_proj(gelu_tanh(c_fc(x))). On ROCm bf16 (default; SDML_FUSED_GELU_GEMM=0 turns it off): the c_fc forward
    and the c_proj input gradient on gemm_bf16.hip with the GELU / GELU' fused into their epilogues (no standalone
    GELU passes), the other two on the hand NT kernel too (SDML_GPT2_GEMM=lib: hipBLASLt). Round 4, one MI355X, GPT-2
    step at 16 x 1024 tokens, the other two on hipBLASLt: 21.82 vs
    21.79 ms with library GEMMs + the standalone GELU kernels (profiles/r4_gpt2_fused_gelu_ab.jsonl) - the 4-phase
    NT mainloop still trails hipBLASLt's per GEMM (99.5 vs 76.7 us at c_fc), the fusion pays the difference back.
    (Round 3, before the 4-phase loop: fused c_fc 124.5 us vs 77 + GELU, so it was off.)"""
    if (x.is_cuda and x.dtype == torch.bfloat16 and w1.dtype == torch.bfloat16 and b1 is not None
            and b2 is not None and (_HAND or os.environ.get("SDML_FUSED_GELU_GEMM", "1") == "1")):
        T, C = x.numel() // x.shape[-1], x.shape[-1]
        k = kernels()
        if (k.gemm_bf16_supported(T, w1.shape[0], C, C, C, False)
                and k.gemm_bf16_supported(T, w2.shape[1], w2.shape[0], w2.shape[0], w2.shape[1], True)
                and x.stride(-1) == 1):
            return _MLPFn.apply(x, w1, b1, w2, b2)
    from .transformer import gelu

    return linear(gelu(linear(x, w1, b1)), w2, b2)


def _wgrad_ok(g2, x2, gw) -> bool:
    return (g2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and gw.dtype == torch.bfloat16
            and g2.stride(-1) == 1 and x2.stride(-1) == 1 and gw.is_contiguous()
            and g2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0
            and kernels().wgrad_bf16_supported(gw.shape[0], gw.shape[1], g2.shape[0]))


def _padded(t, rows):
    """``t`` [V, C] (a parameter or its .grad, inside FlatParams' row-padded storage) as the [rows, C] matrix."""
    C = t.shape[1]
    if (not t.is_contiguous() or t.untyped_storage().nbytes() < (t.storage_offset() + rows * C) * t.element_size()):
        return None
    return t.as_strided((rows, C), (C, 1))


def _w_padded(w):
    """The lm_head weight as its padded [Vp, C] matrix, cached on the parameter (the same storage every step)."""
    rows = getattr(w, "_sdml_rows_padded", 0)
    if rows < w.shape[0]:
        return None
    wp = getattr(w, "_sdml_wpad", None)
    if wp is None or wp.data_ptr() != w.data_ptr() or wp.shape[0] != rows:
        wp = _padded(w, rows)
        w._sdml_wpad = wp
    return wp


class _LMHeadFn(torch.autograd.Function):
    """GPT-2's untied vocabulary head, logits = x W^T (no bias), on the hand-written bf16 kernels.

    The vocabulary (50257) is not a multiple of 8, so W lives in FlatParams' row-padded storage (models/gpt2.py
    ``flat_row_multiple``): the [Vp = 50304, 768] matrix in place, rows past V zero in the weight and in its
    gradient. All three GEMMs then run at Vp: the forward (NT, N = Vp) writes [T, Vp] logits whose pad columns are
    exact zeros and returns the [T, V] view (row stride Vp); the cross-entropy kernel reads that view and writes
    dlogits with the same row stride, zeroing the pad columns (transformer.hip); the input gradient is dlogits W as
    NT against the padded W^T (K = Vp) and the weight gradient dlogits^T x accumulates into the padded gradient
    (its pad rows get exact zeros, so SGD keeps them zero). The results on the V real columns are those of the
    unpadded GEMMs (the pad terms are products with zeros). Reference Linear layers: /root/reference/
    simple_distributed.py:63-64, :75-77; BASELINE config 5 (the lm_head was round 5's last library GEMM)."""

    @staticmethod
    def forward(ctx, x, w):
        wp = _w_padded(w)
        V, C = w.shape
        x2 = x.reshape(-1, C)
        y, _ = kernels().gemm_bf16(x2, wp, None, False, EPI_STORE)
        ctx.save_for_backward(x2)
        ctx.w, ctx.in_shape = w, x.shape
        return y.narrow(1, 0, V).view(*x.shape[:-1], V)

    @staticmethod
    def backward(ctx, gy):
        (x2,) = ctx.saved_tensors
        w = ctx.w
        V, C = w.shape
        wp = _w_padded(w)
        Vp = wp.shape[0]
        g2 = gy.reshape(-1, V)
        T = g2.shape[0]
        gp = None
        if (g2.stride(-1) == 1 and (T == 1 or g2.stride(0) == Vp)
                and g2.untyped_storage().nbytes() >= (g2.storage_offset() + T * Vp) * g2.element_size()):
            gp = g2.as_strided((T, Vp), (Vp, 1))  # the cross-entropy's padded dlogits (pad columns zero)
        if gp is None:  # an unpadded gradient (another loss): pad a copy
            gp = torch.zeros((T, Vp), dtype=g2.dtype, device=g2.device)
            gp[:, :V] = g2
        wpt = _w_t(wp) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:  # (first: on the side stream it runs beside the input gradient)
            gpad = _padded(w.grad, Vp) if w.grad is not None else None
            if gpad is not None and _wgrad_ok(gp, x2, gpad):
                _wgrad_launch(gp, x2, gpad, None)
            else:
                gw = gp[:, :V].t() @ x2
        dx = None
        if ctx.needs_input_grad[0]:
            dx, _ = kernels().gemm_bf16(gp, wpt, None, False, EPI_STORE)
            dx = dx.view(ctx.in_shape)
        return dx, gw


def lm_head(x, w):
    """logits = x W^T (GPT-2's vocabulary head): the padded hand-written path when W sits in row-padded storage on
    ROCm bf16 (see _LMHeadFn), else the plain Linear."""
    if (_HAND and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(-1) == 1
            and _w_padded(w) is not None):
        wp = _w_padded(w)
        k = kernels()
        T, C = x.numel() // x.shape[-1], x.shape[-1]
        Vp = wp.shape[0]
        if (k.gemm_bf16_supported(T, Vp, C, C, C, False) and k.gemm_bf16_supported(T, C, Vp, Vp, Vp, False)):
            return _LMHeadFn.apply(x, w)
    return linear(x, w)


def linear(x, w, b=None):
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        return _LinearFn.apply(x, w, b)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """nn.Linear (same parameter names and init) with the fused-gradient backward on ROCm bf16."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
