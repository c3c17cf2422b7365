"""Fused ops: gfx950 HIP kernels on ROCm devices, PyTorch fp32 reference on CPU.

A CUDA(ROCm) tensor ALWAYS goes to the HIP kernel extension; if it is missing this raises
(no silent fallback to PyTorch on the GPU). CPU tensors use ``ops.reference``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .._native import kernels
from . import reference as ref


def _k():
    return kernels()


def linear_relu_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """relu(x @ w.T + b); x [M,K], w [N,K] (nn.Linear layout), b [N]."""
    if x.is_cuda:
        return _k().linear_fwd_f32(x, w, b, True)
    return ref.linear_relu_fwd(x, w, b)


PIXEL_SCALE = 1.0 / 255.0  # torchvision ToTensor(): uint8 pixel k -> k / 255


def pixels_to_float(x: torch.Tensor) -> torch.Tensor:
    """uint8 pixels -> float32 in [0, 1] exactly as ``ToTensor()`` (the reference's transform,
    /root/reference/simple_distributed.py:87-88); float input passes through."""
    return x.to(torch.float32).div_(255.0) if x.dtype == torch.uint8 else x


class PlaneCache:
    """The uint8 first layer's weight as zero-padded fp16 planes [2][N][Kp] of W * 2^8 (hi + lo
    is W to within one fp32 ulp, csrc/kernels/u8_planes.h).

    The forward needs them every step; instead of a split launch per step, the fused SGD step
    writes them from the weights it has just updated (ops/optim.py, ``add_plane_cache``). The
    cache is valid for the parameter values identified by ``(weight._version, flat.param_epoch)``:
    an optimizer step bumps the epoch and re-validates it, any torch in-place write to the weight
    (checkpoint load, ...) bumps the version and invalidates it (the forward then re-splits)."""

    def __init__(self, weight: torch.Tensor):
        n, k = weight.shape
        self.planes = torch.zeros(int(_k().u8_fwd_planes()), n, int(_k().u8_fwd_kpad(k)), dtype=torch.int16,
                                  device=weight.device)
        self.token = None

    @staticmethod
    def token_of(weight: torch.Tensor, epoch: int):
        return (weight.data_ptr(), weight._version, epoch)


def relu_bits(y: torch.Tensor) -> torch.Tensor:
    """int32 [M, N/32] ReLU mask of y [M, N]: bit n % 32 of word n // 32 is (y[m, n] > 0) - the layout the
    uint8 kernels write (mask_out) and the factored weight gradient reads."""
    M, N = y.shape
    sh = torch.arange(32, device=y.device, dtype=torch.int64)
    w = ((y > 0).view(M, N // 32, 32).to(torch.int64) << sh).sum(-1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def relu_bits_unpack(mask: torch.Tensor) -> torch.Tensor:
    """float 0/1 [M, 32 * words] from :func:`relu_bits`' layout."""
    sh = torch.arange(32, device=mask.device, dtype=torch.int64)
    w = mask.to(torch.int64) & 0xFFFFFFFF
    return ((w.unsqueeze(-1) >> sh) & 1).view(mask.shape[0], -1).to(torch.float32)


def linear_relu_fwd_u8(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, cache: Optional[PlaneCache] = None,
                       epoch: int = 0, mask_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu(ToTensor(x) @ w.T + b) for uint8 pixels x [M,K]: on ROCm the /255 is folded into the
    GEMM's epilogue and each pixel byte is exact in fp16 against two fp16 weight planes (2 MFMAs/product). With a
    ``cache`` (and the flat buffer's ``epoch``) the weight planes are reused when still current.
    ``mask_out`` (int32 [M, N/32]): also receives the output's ReLU bits (:func:`relu_bits`)."""
    if x.is_cuda:
        k = _k()
        # per-wave output maxima: the bound of the next layer's two-plane split (no inf-norm pass over y)
        wm = torch.empty(int(k.u8_fwd_wmax_slots(x.shape[0], w.shape[0])), device=x.device, dtype=torch.float32)
        if cache is None:
            y = k.linear_fwd_u8(x, w, b, True, PIXEL_SCALE, None, False, mask_out, wm)
        else:
            tok = PlaneCache.token_of(w, epoch)
            y = k.linear_fwd_u8(x, w, b, True, PIXEL_SCALE, cache.planes, cache.token == tok, mask_out, wm)
            cache.token = tok
        y._sdml_wmax = wm
        return y
    y = ref.linear_relu_fwd(pixels_to_float(x), w, b)
    if mask_out is not None:
        mask_out.copy_(relu_bits(y))
    return y


def relu_head_u8_supported(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> bool:
    """Whether :func:`linear_relu_head_u8` runs as ONE fused launch for these shapes (ROCm)."""
    return bool(x.is_cuda and x.dtype == torch.uint8 and x.dim() == 2 and x.is_contiguous()
                and x.data_ptr() % 16 == 0
                and _k().u8_fwd_head_supported(x.shape[0], w1.shape[0], x.shape[1], w2.shape[0]))


def linear_relu_head_u8(x, w1, b1, cache: PlaneCache, epoch: int, w2, b2, target, gw2, gb2, loss_scale: float, stats,
                        stats_init: bool, dl_out, mask_out, defer: bool = False):
    """Training step of a uint8-fed hidden layer AND the classifier head in one launch (ROCm:
    mlp_u8.hip u8_fwd_head; h = relu(ToTensor(x) @ w1.T + b1) never leaves the chip). Writes the head's
    factored boundary gradient dl = loss_scale (softmax - onehot) into ``dl_out`` [M, C] and h's ReLU
    bits into ``mask_out`` [M, N/32]; accumulates gw2/gb2 and (loss sum, correct) into ``stats``
    (overwritten with ``stats_init``). Returns (dl bounds, pending): ``pending`` (with ``defer``) is the
    head's deferred slab reduction for :func:`linear_wgrad_u8_dl`'s ``head_pending``. The bounds
    bound |dl @ w2| per block (the weight gradient's dz scale)."""
    if x.is_cuda:
        tok = PlaneCache.token_of(w1, epoch)
        out = _k().linear_relu_head_u8(x, w1, b1, PIXEL_SCALE, cache.planes, cache.token == tok, w2, b2, target,
                                       gw2, gb2, float(loss_scale), stats, bool(stats_init), dl_out, mask_out,
                                       bool(defer))
        cache.token = tok
        return out
    h = linear_relu_fwd_u8(x, w1, b1, mask_out=mask_out)
    with torch.no_grad():
        loss, correct, dl = ref.linear_logsoftmax_nll_dl(h, w2, b2, target, gw2, gb2, loss_scale)
    _put_stats(stats, loss, correct, stats_init)
    dl_out.copy_(dl)
    return None, None


def linear_wgrad_u8(x: torch.Tensor, gz: torch.Tensor, gw: torch.Tensor, gb: Optional[torch.Tensor],
                    amax: Optional[torch.Tensor] = None) -> None:
    """gw += gz.T @ ToTensor(x), gb += sum(gz) for uint8 pixels x (first layer: no input grad).

    ROCm: gz enters the kernel as fp16 planes scaled from a bound on |gz|: ``amax`` (any float
    tensor whose max bounds |gz|), else the bounds the fused head attached to the dx it returned
    (:func:`linear_logsoftmax_nll`) or the per-wave maxima of the x2 GEMM that produced it, else a torch
    amax of gz."""
    if x.is_cuda:
        if amax is None:  # the head's per-block bounds, or the producing GEMM's per-wave maxima (x2 engine)
            amax = getattr(gz, "_sdml_amax", None)
            if amax is None:
                amax = getattr(gz, "_sdml_wmax", None)
        _k().linear_wgrad_u8(x, gz, gw, gb, PIXEL_SCALE, amax)
        return
    gw += gz.t() @ pixels_to_float(x)
    if gb is not None:
        gb += gz.sum(0)


def linear_wgrad_u8_dl(x, dl, w2, h, gw, gb, amax: Optional[torch.Tensor] = None, head_pending=None,
                       sgd=None, groups=None) -> bool:
    """First-layer weight gradient from the FACTORED boundary gradient: with dz = (dl @ w2) * (h > 0)
    (dl [M, C] the head's factor, w2 [C, N] the head weight, h [M, N] this layer's ReLU output - or its
    ReLU bits, int32 [M, N/32] (:func:`relu_bits`), which is all that is read),
    gw += dz.T @ ToTensor(x), gb += sum(dz). On ROCm dz is expanded inside the weight-gradient kernel
    (never written to memory); with the same ``amax`` (a bound on |dz|, see :func:`linear_wgrad_u8`)
    bit-identical to :func:`head_dx_from_dlogits` + :func:`linear_wgrad_u8`; without it the bounds the
    fused head attached to the ``dl`` it returned, else each workgroup bounds dz by its rows'
    max sum |dl| times max |w2| (a dl received over the network carries no attribute).
    ``head_pending``: a head reduction deferred by :func:`linear_logsoftmax_nll_dl`, run in the same
    launch as this one's slab reduction (or before it, on the paths without one).
    ``sgd`` (with ``head_pending``; ops.optim.FusedSGD.fused_args): these are the step's last
    gradients - apply the optimizer step inside the same launch. Returns True if it was applied (the
    caller then commits it with FusedSGD.commit_fused instead of stepping).
    ``groups`` = (g_first, g_count, blocks): only hidden units [64 g_first, 64 (g_first + g_count)) of gw/gb,
    in ~``blocks`` row splits (no ``sgd``): the data-parallel step computes the gradient in two such ranges
    so the first range's all-reduce runs under the second range's kernel (parallel/pipeline.py)."""
    if x.is_cuda:
        if amax is None:
            amax = getattr(dl, "_sdml_amax", None)
        return bool(_k().linear_wgrad_u8_dl(x, dl, w2, h, gw, gb, PIXEL_SCALE, amax, head_pending, sgd,
                                            None if groups is None else tuple(int(g) for g in groups)))
    if head_pending is not None:
        head_pending.run()
    with torch.no_grad():
        mask = relu_bits_unpack(h) if h.dtype == torch.int32 else (h > 0).to(dl.dtype)
        dz = (dl @ w2) * mask
        if groups is not None:
            lo, n = 64 * int(groups[0]), 64 * int(groups[1])
            dz = dz[:, lo:lo + n]
            gw, gb = gw[lo:lo + n], gb[lo:lo + n]
        gw += dz.t() @ pixels_to_float(x)
        gb += dz.sum(0)
    return False


def linear_fwd(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    if x.is_cuda:
        return _k().linear_fwd_f32(x, w, b, False)
    return ref.linear_fwd(x, w, b)


def linear_relu_bwd(x, y, gy, w, gw, gb, need_dx: bool, gy_masked: bool = False, mask_dx: bool = False):
    """Backward of y = relu(x @ w.T + b): accumulates gw += gz.T @ x, gb += sum(gz) with
    gz = gy * (y > 0) (``gy_masked``: gy already is gz, skip the mask); returns gz @ w when
    need_dx, times (x > 0) when ``mask_dx`` (the producing layer's ReLU backward, fused)."""
    if x.is_cuda:
        return _k().linear_bwd_f32(x, y, gy, w, gw, gb, need_dx, not gy_masked, mask_dx)
    dx = ref.linear_relu_bwd(x, y, gy, w, gw, gb, need_dx)
    if dx is not None and mask_dx:
        dx = dx * (x > 0).to(dx.dtype)
    return dx


# ---- fp32-accurate hidden layers on two fp16 planes (csrc/kernels/gemm_f16x2.hip) -------------------
# Every operand is split ONCE into fp16 planes (hi, lo of x * 2^s) and each product costs 3 fp16 MFMAs
# (the bf16x3 engine: 6, with the split redone inside every GEMM). The planes of a layer's input serve its
# forward (A operand) and its weight gradient (B operand); the weight's planes serve forward and input
# gradient. Bounds for the splits come from the producing kernel where it has one (the GEMM epilogues'
# per-wave maxima ``_sdml_wmax``, the head's per-block bounds ``_sdml_amax``), else from an inf-norm pass.
# SDML_F32_GEMM=x3 keeps the bf16x3 engine (A/B).

_X2_MIN_ROWS = 2048
_X2_DX_NT = __import__("os").environ.get("SDML_X2_DX", "nt") != "nn"  # A/B: SDML_X2_DX=nn (w planes, NN kernel)


def _x2_env_ok() -> bool:
    import os

    return os.environ.get("SDML_F32_GEMM", "x2") not in ("x3", "mfma")


def x2_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether the layer y = x @ w.T runs on the two-plane engine (ROCm fp32, large enough shapes)."""
    if not (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2
            and x.is_contiguous() and w.is_contiguous() and x.shape[0] >= _X2_MIN_ROWS and _x2_env_ok()):
        return False
    M, K = x.shape
    N = w.shape[0]
    k = _k()
    return bool(K % 64 == 0 and N % 64 == 0 and k.x2_gemm_supported(M, N, K, False)
                and k.x2_gemm_supported(M, K, N, True))


def _bound_of(t: torch.Tensor) -> torch.Tensor:
    b = getattr(t, "_sdml_wmax", None)
    if b is None:
        b = getattr(t, "_sdml_amax", None)
    if b is None:
        b = torch.linalg.vector_norm(t, float("inf")).reshape(1)
    return b


def carry_bounds(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """Keep the bound attributes of ``src`` on ``dst`` (a reshaped view / same-data alias of it)."""
    if dst is not src:
        for a in ("_sdml_wmax", "_sdml_amax"):
            v = getattr(src, a, None)
            if v is not None:
                setattr(dst, a, v)
    return dst


def x2_split(t: torch.Tensor):
    """(planes int16 [2, rows, cols], dequantisation scale [1]) of an fp32 matrix."""
    return _k().x2_split(t, _bound_of(t))


def linear_relu_fwd_x2(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], relu: bool = True):
    """relu(x @ w.T + b) on the two-plane engine. Returns (y, planes) with planes = (x planes, x scale,
    w planes, w scale) for :func:`linear_relu_bwd_x2`; y carries its per-wave maxima for the next split."""
    k = _k()
    xp, sx = x2_split(x)
    wn = torch.linalg.vector_norm(w, float("inf")).reshape(1)
    wp, sw = k.x2_split(w, wn)
    y, wm = k.x2_gemm(xp, sx, wp, sw, False, b, relu, None, True)
    y._sdml_wmax = wm
    # the input gradient dz @ w runs as an NT GEMM against w^T's planes (the 4-phase NT kernel)
    wtp, swt = k.x2_split_t(w, wn) if _X2_DX_NT else (wp, sw)
    return y, (xp, sx, wtp, swt)


def linear_relu_bwd_x2(x: torch.Tensor, gz: torch.Tensor, gw, gb, planes, need_dx: bool, mask_dx: bool):
    """Backward of y = relu(x @ w.T + b) given gz = dL/d(pre-activation) (already masked): gw += gz.T @ x,
    gb += sum(gz) and, when ``need_dx``, returns gz @ w (times (x > 0) with ``mask_dx``), all from planes."""
    xp, sx, wp, sw = planes
    gp, sg = x2_split(gz.contiguous())
    dx = None
    if need_dx:
        dx, wm = _k().x2_gemm(gp, sg, wp, sw, not _X2_DX_NT, None, False, x if mask_dx else None, True)
        dx._sdml_wmax = wm
    _k().x2_wgrad_(gp, sg, xp, sx, gw, gb)
    return dx


def _put_stats(stats, loss, correct, init: bool):
    if init:
        stats[0] = loss
        stats[1] = correct
    else:
        stats[0] += loss
        stats[1] += correct


def linear_logsoftmax_nll(x, w, b, target, gw, gb, scale: float, need_dx: bool, stats=None, mask_dx: bool = False,
                          stats_init: bool = False):
    """Fused classifier head: z = x @ w.T + b -> log_softmax -> NLL (sum) and, when grads are
    given, the full backward (gw/gb accumulated, dx returned) scaled by ``scale``.

    Returns (loss_sum, correct, dx). With ``stats`` (a float32 [2] tensor) the loss sum and
    correct count are ACCUMULATED into it in-kernel (``stats_init``: overwrite it, so it needs no
    zero-fill beforehand) and (None, None, dx) is returned.
    ``mask_dx``: dx *= (x > 0) (fused ReLU backward of the stage that produced x)."""
    if x.is_cuda:
        st, dx, amax = _k().head_logsoftmax_nll_f32(x, w, b, target, gw, gb, float(scale), need_dx, stats, mask_dx,
                                                    bool(stats_init))
        if dx is not None and amax is not None:
            dx._sdml_amax = amax  # per-block bounds on |dx|, which linear_wgrad_u8 scales dz's fp16 planes with
        if stats is not None:
            return None, None, dx
        return st[0], st[1], dx
    loss, correct, dx = ref.linear_logsoftmax_nll(x, w, b, target, gw, gb, scale, need_dx)
    if dx is not None and mask_dx:
        dx = dx * (x > 0).to(dx.dtype)
    if stats is not None:
        _put_stats(stats, loss, correct, stats_init)
        return None, None, dx
    return loss, correct, dx


def linear_logsoftmax_nll_dl(x, w, b, target, gw, gb, scale: float, stats, stats_init: bool = False,
                             defer_reduce: bool = False):
    """Training head (fc -> log_softmax -> NLL, backward) whose boundary gradient is returned as its
    rank-C factor ``dl = scale * (softmax - onehot)`` [M, C] instead of ``dx = dl @ w`` [M, K]
    (:func:`head_dx_from_dlogits` rebuilds dx bit-identically wherever ``w`` is held). gw/gb are
    accumulated; loss sum and correct count are accumulated into ``stats`` [2] (overwritten with
    ``stats_init``).

    ``defer_reduce``: return ``(dl, pending)``; on ROCm the head's slab reduction (gw/gb/stats) is
    then left to ``pending`` (None when nothing was deferred), which the caller MUST hand to
    :func:`linear_wgrad_u8_dl` (``head_pending``: both reductions in one launch) or run itself
    (``pending.run()``) before it reads gw/gb/stats."""
    if x.is_cuda:
        dl, amax, pending = _k().head_logsoftmax_nll_dl_f32(x, w, b, target, gw, gb, float(scale), stats,
                                                             bool(stats_init), bool(defer_reduce))
        if amax is not None:
            dl._sdml_amax = amax  # per-block bounds on |dl @ w| (linear_wgrad_u8_dl's dz bound)
        return (dl, pending) if defer_reduce else dl
    with torch.no_grad():
        loss, correct, dl = ref.linear_logsoftmax_nll_dl(x, w, b, target, gw, gb, scale)
    _put_stats(stats, loss, correct, stats_init)
    return (dl, None) if defer_reduce else dl


def pooled_head_xent(y, w, b, target, gw, gb, scale: float, stats, stats_init: bool = False):
    """Training head of a convolutional stage (ResNet's last layer): global average pool of ``y``
    ([N, C, H, W], channels-last memory) -> Linear(w, b) -> log_softmax -> NLL (sum), with the whole backward:
    gw/gb accumulated (scaled by ``scale``), loss sum / correct count into ``stats`` [2] (added; overwritten
    with ``stats_init``). Returns dy (the gradient w.r.t. ``y``, same layout). ROCm only:
    csrc/kernels/head_pool.hip (one launch + one fixed-order reduction)."""
    N, C, H, W = y.shape
    yl = y.permute(0, 2, 3, 1)  # channels-last memory as [N, H, W, C]: contiguous
    if not yl.is_contiguous():
        yl = yl.contiguous()
    dy = _k().head_pool_xent(yl.view(N, H * W, C), w.detach(), b.detach(), target, gw, gb, float(scale), stats,
                             bool(stats_init))
    return dy.view(N, H, W, C).permute(0, 3, 1, 2)


def pooled_head_ok(y, w) -> bool:
    return bool(y.is_cuda and y.dim() == 4 and y.dtype in (torch.bfloat16, torch.float32) and w.dtype == y.dtype
                and w.is_contiguous() and w.data_ptr() % 16 == 0 and y.data_ptr() % 16 == 0
                and _k().head_pool_supported(y.shape[0], y.shape[2] * y.shape[3], y.shape[1], w.shape[0]))


def head_dx_from_dlogits(dl, w, x, mask: bool = True):
    """Boundary gradient from its factor: ``(dl @ w) * (x > 0)`` (the ReLU backward of the stage
    that produced ``x``, fused), with the fused head's exact arithmetic on ROCm."""
    if dl.is_cuda:
        return _k().head_dx_from_dl(dl, w, x, bool(mask))
    with torch.no_grad():
        dx = dl @ w
    return dx * (x > 0).to(dx.dtype) if mask else dx


def sgd_momentum_(p, g, buf, lr: float, momentum: float, dampening: float = 0.0, weight_decay: float = 0.0,
                  nesterov: bool = False, first: bool = False, zero_grad: bool = False, planes=None):
    """In-place SGD step; with ``zero_grad`` the kernel also clears ``g`` after reading it.
    ``planes = (cache_tensor, offset, rows, K)``: also write that weight's fp16 plane cache from the
    updated values (ROCm only)."""
    if p.is_cuda:
        if planes is not None:
            t, off, rows, k = planes
            _k().sgd_momentum_(p, g, buf, float(lr), float(momentum), float(dampening), float(weight_decay),
                               bool(nesterov), bool(first), bool(zero_grad), t, int(off), int(rows), int(k))
        else:
            _k().sgd_momentum_(p, g, buf, float(lr), float(momentum), float(dampening), float(weight_decay),
                               bool(nesterov), bool(first), bool(zero_grad))
        return
    ref.sgd_momentum_(p, g, buf, lr, momentum, dampening, weight_decay, nesterov, first)
    if zero_grad:
        g.zero_()


def sgd_momentum_mixed_(master, p, g, buf, lr: float, momentum: float, dampening: float = 0.0,
                        weight_decay: float = 0.0, nesterov: bool = False, first: bool = False,
                        zero_grad: bool = False):
    """SGD on fp32 ``master`` weights from low-precision grads ``g``; writes ``p`` = bf16(master)."""
    if master.is_cuda:
        _k().sgd_momentum_mixed_(master, p, g, buf, float(lr), float(momentum), float(dampening),
                                 float(weight_decay), bool(nesterov), bool(first), bool(zero_grad))
        return
    ref.sgd_momentum_(master, g.float(), buf, lr, momentum, dampening, weight_decay, nesterov, first)
    p.copy_(master)
    if zero_grad:
        g.zero_()


# ---- reference CNN: one launch per stage pass (csrc/kernels/ref_cnn.hip) --------------------
# Dropout seeds: ``seed`` (host, per pass) combined with ``ctr`` (optional int64 device step
# counter, advanced inside captured hipGraphs) as ops.reference.effective_seed.
def ref_cnn_stage0_fwd(x, conv1, conv2, seed: int, p: float, drop: bool, sample0: int = 0, ctr=None,
                       save: bool = False):
    """Network1 (conv1-pool-relu-conv2-dropout2d-pool-relu-flatten) -> (out [B, 320], saved).
    ``save`` (training) also returns what :func:`ref_cnn_stage0_bwd` needs."""
    if x.is_cuda:
        out, z1, idx = _k().ref_cnn_stage0_fwd(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, seed, ctr,
                                               sample0, p, drop, save)
        return out, ((z1, idx) if save else None)
    seed_e = ref.effective_seed(seed, ctr)
    with torch.no_grad():
        out = ref.ref_cnn_stage0(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, seed_e, sample0, p, drop)
    return out, (None if not save else ())


def ref_cnn_stage0_bwd(x, conv1, conv2, out, gout, saved, seed: int, p: float, drop: bool, sample0: int = 0,
                       ctr=None):
    """Accumulates conv1/conv2 weight and bias grads from the forward's output/saved state."""
    if x.is_cuda:
        z1, idx = saved
        _k().ref_cnn_stage0_bwd(x, conv2.weight, out, gout.contiguous(), z1, idx, seed, ctr, sample0, p, drop,
                                conv1.weight.grad, conv1.bias.grad, conv2.weight.grad, conv2.bias.grad)
        return
    seed = ref.effective_seed(seed, ctr)
    ps = [conv1.weight, conv1.bias, conv2.weight, conv2.bias]
    leaves = [t.detach().requires_grad_(True) for t in ps]
    with torch.enable_grad():
        y = ref.ref_cnn_stage0(x, *leaves, seed, sample0, p, drop)
        gs = torch.autograd.grad(y, leaves, gout)
    for t, g in zip(ps, gs):
        t.grad.add_(g)


def ref_cnn_stage1(x, fc1, fc2, target, seed: int, p: float, drop: bool, scale: float, stats, train: bool,
                   sample0: int = 0, ctr=None):
    """Network2 + NLL: stats[0] += sum loss, stats[1] += correct; when ``train`` accumulates
    fc1/fc2 grads of ``scale * sum loss`` and returns dL/dx."""
    if x.is_cuda:
        g = (fc1.weight.grad, fc1.bias.grad, fc2.weight.grad, fc2.bias.grad) if train else (None,) * 4
        return _k().ref_cnn_stage1(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, target, seed, ctr, sample0, p,
                                   drop, scale, stats, *g)
    seed = ref.effective_seed(seed, ctr)
    ps = [fc1.weight, fc1.bias, fc2.weight, fc2.bias]
    leaves = [t.detach().requires_grad_(train) for t in ps]
    xx = x.detach().requires_grad_(train)
    with torch.set_grad_enabled(train):
        logp = ref.ref_cnn_stage1_logp(xx, *leaves, seed, sample0, p, drop)
        loss = F.nll_loss(logp, target, reduction="sum")
    stats[0] += loss.detach()
    stats[1] += (logp.argmax(1) == target).sum().to(stats.dtype)
    if not train:
        return None
    gs = torch.autograd.grad(loss * scale, [xx] + leaves)
    for t, g in zip(ps, gs[1:]):
        t.grad.add_(g)
    return gs[0]


def mlp_small_step_args(fc1, fc2, optimizer):
    """The parameter / momentum views :func:`mlp_small_step` takes, built once per engine (the flat
    buffers never move): per step only the batch-dependent arguments cross the binding."""
    mv = [optimizer.buffer_view(p) for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias)]
    return (fc1.weight, fc1.bias, fc2.weight, fc2.bias, *mv)


def mlp_small_step(x, target, fc1, fc2, optimizer, scale: float, stats, args=None) -> bool:
    """ROCm: the whole 784-128-10 training step (both stages' forward, loss, backward and the SGD update
    of fc1/fc2, torch.optim.SGD semantics) in two launches (mlp_small.hip) for batches of up
    to ``mlp_small_step_max_batch()`` rows. ``stats`` [2] receives (loss sum, correct). Returns False
    when it did not run (the caller then takes the multi-kernel path)."""
    k = _k()
    if x.shape[0] > k.mlp_small_step_max_batch():
        return False
    o = optimizer
    if args is None:
        args = mlp_small_step_args(fc1, fc2, optimizer)
    return bool(k.mlp_small_step(x, target, *args, float(o.lr), float(o.momentum), float(o.dampening),
                                 float(o.weight_decay), bool(o.nesterov), o.steps == 0, float(scale), stats))


def ref_cnn_step_args(s0, s1, optimizer):
    """The parameter / momentum views :func:`ref_cnn_step` takes, built once per engine (the flat buffers never
    move; rebuilding the 8 momentum views was ~40 % of the step's host time at B = 60)."""
    params = [s0.conv1.weight, s0.conv1.bias, s0.conv2.weight, s0.conv2.bias,
              s1.fc1.weight, s1.fc1.bias, s1.fc2.weight, s1.fc2.bias]
    return [p.data for p in params], [optimizer.buffer_view(p) for p in params]


def ref_cnn_step(x, target, s0, s1, optimizer, scale: float, stats, ctr, seed0: int, seed1: int, args=None) -> None:
    """ROCm: the reference CNN's whole training step - stage 0 forward, stage 1 forward + NLL + backward,
    stage 0 backward and torch.optim.SGD on all 8 tensors - in two launches (ref_cnn.hip: one workgroup per
    sample, then a fixed-order reduction of the per-sample records that applies the update). ``stats`` [2]
    receives (loss sum, correct); the dropout counter ``ctr`` is advanced on the device."""
    o = optimizer
    params, bufs = args if args is not None else ref_cnn_step_args(s0, s1, optimizer)
    p0, p1 = float(s0.conv2_drop.p), float(s1.p)
    _k().ref_cnn_step(x, target, params, bufs, int(seed0), int(seed1), ctr, p0, p0 > 0, p1, p1 > 0,
                      float(scale), float(o.lr), float(o.momentum), float(o.dampening), float(o.weight_decay),
                      bool(o.nesterov), o.steps == 0, stats)
