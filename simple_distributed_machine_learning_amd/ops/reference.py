"""Plain-PyTorch fp32 reference implementations of every fused op.

They define the exact semantics the HIP kernels (csrc/kernels/*.hip) must reproduce and are
what the numerics tests compare against. They also serve the CPU (Gloo) path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def linear_relu_fwd(x, w, b):
    return torch.relu(x @ w.t() + b)


def linear_relu_bwd(x, y, gy, w, gw: Optional[torch.Tensor], gb: Optional[torch.Tensor], need_dx: bool):
    gz = gy * (y > 0).to(gy.dtype)
    if gw is not None:
        gw += gz.t() @ x
    if gb is not None:
        gb += gz.sum(0)
    return gz @ w if need_dx else None


def linear_fwd(x, w, b):
    return x @ w.t() + (b if b is not None else 0)


def linear_logsoftmax_nll(x, w, b, target, gw, gb, scale: float, need_dx: bool):
    z = x @ w.t() + b
    lp = F.log_softmax(z, dim=1)
    loss = -lp.gather(1, target.view(-1, 1)).sum()
    correct = (lp.argmax(1) == target).sum()
    dx = None
    if gw is not None or need_dx:
        dz = lp.exp()
        dz[torch.arange(z.shape[0]), target] -= 1.0
        dz *= scale
        if gw is not None:
            gw += dz.t() @ x
        if gb is not None:
            gb += dz.sum(0)
        if need_dx:
            dx = dz @ w
    return loss, correct, dx


def linear_logsoftmax_nll_dl(x, w, b, target, gw, gb, scale: float):
    """Training head whose boundary gradient is returned as its factor dl = scale * (softmax - onehot)
    (dx = dl @ w); gw/gb accumulated. Returns (loss_sum, correct, dl)."""
    z = x @ w.t() + b
    lp = F.log_softmax(z, dim=1)
    loss = -lp.gather(1, target.view(-1, 1)).sum()
    correct = (lp.argmax(1) == target).sum()
    dl = lp.exp()
    dl[torch.arange(z.shape[0]), target] -= 1.0
    dl *= scale
    gw += dl.t() @ x
    gb += dl.sum(0)
    return loss, correct, dl


def sgd_momentum_(p, g, buf, lr: float, momentum: float, dampening: float = 0.0, weight_decay: float = 0.0,
                  nesterov: bool = False, first: bool = False):
    """torch.optim.SGD semantics (first step: buf = g, no dampening)."""
    d = g if weight_decay == 0 else g + weight_decay * p
    if momentum != 0:
        if first:
            buf.copy_(d)
        else:
            buf.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d + momentum * buf if nesterov else buf
    p.add_(d, alpha=-lr)


def cross_entropy_fwd_bwd(logits, target, scale: float, ignore_index: int = -100):
    """Returns (loss_sum, correct, count, dlogits) with dlogits = scale * (softmax - onehot)."""
    z = logits.float()
    lse = torch.logsumexp(z, dim=1, keepdim=True)
    valid = target != ignore_index
    t = target.clamp_min(0)
    loss = (lse.squeeze(1) - z.gather(1, t.view(-1, 1)).squeeze(1))[valid].sum()
    correct = ((z.argmax(1) == target) & valid).sum()
    g = torch.exp(z - lse)
    g[torch.arange(z.shape[0]), t] -= 1.0
    g *= scale
    g[~valid] = 0
    return loss, correct, int(valid.sum()), g.to(logits.dtype)


def layernorm_fwd(x, w, b, eps: float = 1e-5):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def gelu_tanh(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


# ---- reference CNN (ref_cnn.hip) ------------------------------------------------------------
_M64 = (1 << 64) - 1


def dropout_keep_scale(seed: int, sample0: int, n: int, units: int, p: float) -> torch.Tensor:
    """[n, units] float32 dropout multipliers, bit-identical to ref_cnn.hip's counter hash:
    keep iff u(seed, sample0 + i, unit) >= p, kept units scaled by 1/(1-p)."""
    import numpy as np
    if p <= 0.0:
        return torch.ones(n, units)
    a = (np.arange(n, dtype=np.uint64) + np.uint64(sample0) + np.uint64(1))[:, None]
    b = np.arange(units, dtype=np.uint64)[None, :] + np.uint64(7)
    with np.errstate(over="ignore"):
        x = (np.uint64(seed & _M64) ^ (np.uint64(0x9E3779B97F4A7C15) * a) ^ (np.uint64(0xC2B2AE3D27D4EB4F) * b))
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    h = (x & np.uint64(0xFFFFFFFF)) >> np.uint64(8)
    u = h.astype(np.float32) * np.float32(1.0 / 16777216.0)
    keep = u >= np.float32(p)
    sc = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return torch.from_numpy(np.where(keep, sc, np.float32(0.0)).astype(np.float32))


def effective_seed(seed: int, ctr=None) -> int:
    """ref_cnn.hip's eff_seed: seed + 0x9E3779B97F4A7C15 * step_counter (mod 2^64)."""
    c = 0 if ctr is None else int(ctr.reshape(-1)[0])
    return (seed + 0x9E3779B97F4A7C15 * c) & _M64


def ref_cnn_stage0(x, w1, b1, w2, b2, seed: int, sample0: int, p: float, drop: bool):
    """Network1 forward with hash-based Dropout2d (autograd-capable)."""
    z1 = F.relu(F.max_pool2d(F.conv2d(x, w1, b1), 2))
    z2 = F.conv2d(z1, w2, b2)
    if drop:
        z2 = z2 * dropout_keep_scale(seed, sample0, x.shape[0], 20, p).to(z2.device)[:, :, None, None]
    return F.relu(F.max_pool2d(z2, 2)).reshape(-1, 320)


def ref_cnn_stage1_logp(x, w1, b1, w2, b2, seed: int, sample0: int, p: float, drop: bool):
    """Network2 forward (log-probabilities) with hash-based dropout (autograd-capable)."""
    h = F.relu(F.linear(x, w1, b1))
    if drop:
        h = h * dropout_keep_scale(seed, sample0, x.shape[0], 50, p).to(h.device)
    return F.log_softmax(F.linear(h, w2, b2), dim=1)
