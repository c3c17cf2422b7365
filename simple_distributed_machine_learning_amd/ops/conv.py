"""3x3 / stride 1 / pad 1 convolution on channels-last bf16 tensors, backed by the hand-written
implicit-GEMM kernels of csrc/kernels/conv_bf16.hip (forward, input gradient = the forward kernel
with flipped/transposed weights, weight gradient accumulated into ``weight.grad`` in place).

Used by the ResNet-18-style stages (models/resnet.py) when they run in bf16 channels-last: the
twelve stride-1 3x3 convolutions, the one-channel stem, and the stride-2 3x3 / 1x1 shortcut
convolutions (forward, weight gradient and - as four parity-class GEMMs - input gradient), so a bf16
ResNet step launches no MIOpen convolution. Other dtypes/layouts run ``F.conv2d`` on the CPU only: on a GPU
they are refused (``_refuse_library``).
"""
from __future__ import annotations

import weakref

import torch
import torch.nn.functional as F

from .._native import kernels
from . import side_stream


# ResidualLink joins (set False to let autograd add the two gradients of a block input, for A/B tests)
FUSE_RESIDUAL = True


class ResidualLink:
    """Joins the two input gradients of a residual block's input x without an add kernel: the
    residual branch's gradient (through ``grad_tap``) is handed to the main branch's first
    convolution, whose input-gradient epilogue adds it (dx = bf16(conv + addend)).

    The tap is created after the main branch's convolutions in the forward pass, so autograd
    (ready nodes run in decreasing creation order) runs it first. Either order stays correct:
    a convolution that finds no addend marks the link consumed, and a tap that comes later then
    returns its gradient to autograd as usual. ``fused`` counts the joins done in an epilogue."""

    __slots__ = ("addend", "consumed")
    fused = 0

    def __init__(self):
        self.addend = None
        self.consumed = False

    def take(self):
        add, self.addend = self.addend, None
        if add is None:
            self.consumed = True
        else:
            ResidualLink.fused += 1
        return add


class _GradTapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        if link.consumed:
            return g, None
        link.addend = g.contiguous(memory_format=torch.channels_last)
        return None, None


def grad_tap(x: torch.Tensor, link) -> torch.Tensor:
    """x, with its gradient routed through ``link`` (see ResidualLink); identity without a link."""
    if link is None or not x.requires_grad:
        return x
    return _GradTapFn.apply(x, link)


def _take_addend(link):
    return link.take() if link is not None else None


# BNBackLink joins a BatchNorm's backward statistics pass to the convolution whose input gradient is that BatchNorm's
# output gradient dy (ResNet: bn1 -> conv2, and a block's closing BatchNorm -> the next block's conv1 with the residual
# addend fused). Set False for A/B runs.
FUSE_BN_BACK = __import__("os").environ.get("SDML_BN_BACK_FUSE", "1") != "0"


class BNBackLink:
    """Hands a training BatchNorm's backward statistics (per-channel sums of g = dy * relu-mask and g * xhat) to the
    epilogue of the convolution that produces its dy (conv_bf16.hip ``BnBack``), so ``bn_nhwc_bwd`` skips its pass
    over dy and x (batchnorm_nhwc.hip ``bn_partial_kernel<true>``).

    The BatchNorm's forward fills ``args`` (detached x, the saved output when the ReLU mask comes from it, mean, rstd,
    gamma, beta, mask mode); the consuming convolution's backward writes ``part`` for its output and records that
    output's address; the BatchNorm's backward uses ``part`` only when its dy IS that output (so a gradient that
    autograd accumulated from another consumer is never paired with partial sums of one summand).
    ``needs_addend``: the BatchNorm output also feeds a residual branch, so the convolution's output is the whole dy
    only when the branch's gradient was added in its epilogue (ResidualLink). ``fused`` counts the fused passes."""

    __slots__ = ("args", "part", "rows", "dy_ptr", "needs_addend")
    fused = 0

    def __init__(self, needs_addend: bool = False):
        self.args = None
        self.part = None
        self.rows = 0
        self.dy_ptr = None
        self.needs_addend = needs_addend

    def request(self, add):
        """The BatchNorm's saved state for the consumer's dgrad epilogue, or None (then nothing is fused)."""
        if self.args is None or (self.needs_addend and add is None):
            return None
        return self.args

    def fill(self, part, rows, dy):
        self.part, self.rows, self.dy_ptr = part, rows, dy.data_ptr()
        self.args = None

    def take(self, dy):
        """(part, rows) for this dy, or (None, 0); the link is emptied either way."""
        part, rows, ptr = self.part, self.rows, self.dy_ptr
        self.args = self.part = self.dy_ptr = None
        if part is None or ptr != dy.data_ptr():
            return None, 0
        BNBackLink.fused += 1
        return part, rows


def _bn_kwargs(args):
    x, y, mean, rstd, gamma, beta, relu = args
    return dict(bn_x=x, bn_y=y, bn_mean=mean, bn_rstd=rstd, bn_gamma=gamma, bn_beta=beta, bn_relu=relu)


# The kernels' weight layouts (conv3x3_weights_bf16: the forward [Co][9][C] and the flipped / transposed dgrad
# one) depend only on the weight, which is constant within an optimizer step: every micro-batch of a step used
# to re-derive them (16 launches per ResNet-18 step, 0.14 ms of 4.69: profiles/r3_resnet18_bf16_final_kernel_
# stats.txt). They are cached per weight, keyed on (storage, version, WEIGHT_GEN): the fused SGD kernels
# rewrite parameters through raw pointers (no version bump) and so bump WEIGHT_GEN (ops/optim.py); a torch
# in-place write bumps the version. Never used while a hipGraph is being captured (the replays must
# re-derive the layouts from the weights they update). An entry holds a weak reference to its weight: a hit
# requires the very same tensor object (not just a reused id / allocator block of a freed model), and the entry
# is dropped when the weight is freed.
WEIGHT_GEN = [0]
_WCACHE = {}


def _cache_put(cache, w, entry):
    """cache[id(w)] = (weakref to w, *entry); the entry leaves with w."""
    k = id(w)

    def _gone(r, k=k, cache=cache):
        if cache.get(k, (None,))[0] is r:
            cache.pop(k, None)

    cache[k] = (weakref.ref(w, _gone),) + tuple(entry)


def _cache_get(cache, w):
    """The entry stored for exactly this tensor object (without the reference), or None."""
    hit = cache.get(id(w))
    if hit is None or hit[0]() is not w:
        return None
    return hit[1:]
_WCACHE_ON = __import__("os").environ.get("SDML_CONV_WCACHE", "1") != "0"


def bump_weight_generation():
    WEIGHT_GEN[0] += 1
    _WCACHE.clear()


# Every 3x3 weight seen so far keeps one pair of layout buffers across optimizer steps (_KNOWN: id -> (weakref, wt,
# wd or None)). The first layout request of a step re-derives them for ALL live known weights in one launch
# (conv3x3_weights_batched_bf16): a ResNet-18 step made 16 transform launches of ~9 us each, mostly launch
# latency (profiles/r5_resnet18_kernel_stats.txt). Reusing the buffers is safe: a step's backward reads its layouts
# before the optimizer step that bumps WEIGHT_GEN, and the next step's forward rewrites them after it.
_KNOWN = {}


def _known_put(w, wt, wd):
    k = id(w)

    def _gone(r, k=k):
        if _KNOWN.get(k, (None,))[0] is r:
            _KNOWN.pop(k, None)

    _KNOWN[k] = (weakref.ref(w, _gone), wt, wd)


def _weight_layouts(w, need_dgrad: bool):
    K = kernels()
    capturing = torch.cuda.is_current_stream_capturing() or not _WCACHE_ON
    key = (w.data_ptr(), w._version, WEIGHT_GEN[0], tuple(w.shape))
    hit = None if capturing else _cache_get(_WCACHE, w)
    if hit is not None and hit[0] == key and (hit[2] is not None or not need_dgrad):
        return hit[1], hit[2]
    if capturing:
        if need_dgrad:
            return K.conv3x3_weights_bf16(w)
        return K.conv3x3_weight_bf16(w, False), None
    kn = _KNOWN.get(id(w))
    if kn is None or kn[0]() is not w or (need_dgrad and kn[2] is None):
        Co, C = w.shape[0], w.shape[1]
        wt = torch.empty((Co, 9, C), dtype=w.dtype, device=w.device)
        wd = torch.empty((C, 9, Co), dtype=w.dtype, device=w.device) if need_dgrad else None
        _known_put(w, wt, wd)
    # this weight and every other live known weight whose layouts are stale, in one launch
    todo = []
    for k, (ref, wt, wd) in list(_KNOWN.items()):
        ww = ref()
        if ww is None or ww.device != w.device or ww.dtype != w.dtype or not ww.is_contiguous():
            continue
        kk = (ww.data_ptr(), ww._version, WEIGHT_GEN[0], tuple(ww.shape))
        h = _cache_get(_WCACHE, ww)
        if h is not None and h[0] == kk and (h[2] is not None or wd is None):
            continue
        todo.append((ww, wt, wd, kk))
    K.conv3x3_weights_batched_bf16([t[0] for t in todo], [t[1] for t in todo], [t[2] for t in todo])
    for ww, wt, wd, kk in todo:
        _cache_put(_WCACHE, ww, (kk, wt, wd))
    h = _cache_get(_WCACHE, w)
    return h[1], h[2]


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, part=None, link=None, back=None):
        # both layouts in one pass when an input gradient is needed; the dgrad one waits for backward
        wt, ctx.wd = _weight_layouts(w, ctx.needs_input_grad[0])
        K = kernels()
        if not ctx.needs_input_grad[0]:
            ctx.wd = None
        y = K.conv3x3_fwd_bf16(x, wt, part=part)
        ctx.save_for_backward(x)
        ctx.w, ctx.link, ctx.back = w, link, back
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.w
        K = kernels()
        dy = dy.contiguous(memory_format=torch.channels_last)
        gw = None
        late = None  # the side-stream weight gradient, enqueued after the input gradient (side_stream.CONV_WGRAD_AFTER)
        if ctx.needs_input_grad[1]:
            if w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == torch.bfloat16:
                # straight into the flat gradient buffer (SDML_CONV_WGRAD_STREAM=1: on the side stream, beside the input
                # gradient below; ops/side_stream.py)
                g = w.grad
                late = _side_wgrad(lambda: K.conv3x3_wgrad_bf16_(dy, x, g), dy, x, ctx.needs_input_grad[0])
            else:
                gw = torch.zeros_like(w)
                K.conv3x3_wgrad_bf16_(dy, x, gw)
        dx = None
        if ctx.needs_input_grad[0]:
            add = _take_addend(ctx.link)
            req = ctx.back.request(add) if ctx.back is not None else None
            if req is not None:  # dx is the preceding BatchNorm's dy: its backward statistics come from this epilogue
                rows = K.conv_part_rows(dy.shape[0], dy.shape[2], dy.shape[3])
                part = torch.empty(rows * 2 * x.shape[1], device=dy.device, dtype=torch.float32)
                dx = K.conv3x3_fwd_bf16(dy, ctx.wd, add=add, part=part, **_bn_kwargs(req))
                ctx.back.fill(part, rows, dx)
            else:
                dx = K.conv3x3_fwd_bf16(dy, ctx.wd, add=add)
        if late is not None:
            late()
        ctx.wd = ctx.back = None
        return dx, gw, None, None, None


def _side_wgrad(fn, dy, x, dx_follows: bool):
    """Launch a convolution's weight gradient ``fn`` (on the side stream when SDML_CONV_WGRAD_STREAM=1). Returns None
    once launched, or - side stream on, ``CONV_WGRAD_AFTER``, an input gradient to come - a closure the caller runs
    after enqueuing the input gradient: the side stream then waits for an event recorded here, before it, so the two
    still overlap but the input gradient's workgroups reach the CUs first."""
    on = side_stream.CONV_WGRAD_STREAM
    if on and dx_follows and side_stream.CONV_WGRAD_AFTER:
        ev = side_stream.ready_event(dy)
        if ev is not None:
            return lambda: side_stream.launch(fn, dy, x, ready=ev)
    side_stream.launch(fn, dy, x, enabled=on)
    return None


def hip_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    w = conv.weight
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and conv.bias is None
            and tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def _general_dgrad(dy, x, w, st, pd, add=None, back=None):
    """Input gradient of a general_eligible convolution (+ add): stride 2 -> the parity-class GEMM
    kernel (conv_bf16.hip conv_dgrad_s2_kernel); stride-1 1x1 -> the forward kernel on dy with the
    transposed [C][1][Co] weights; stride-1 3x3 -> the forward kernel with the flipped dgrad weights.
    ``back`` (BNBackLink, stride 2): the preceding BatchNorm's backward statistics from the epilogue."""
    K = kernels()
    H, W = x.shape[2], x.shape[3]
    if st == 2:
        req = back.request(add) if back is not None else None
        if req is not None:
            rows = K.conv_dgrad_s2_part_rows(x.shape[0], H, W, w.shape[2], pd)
            part = torch.empty(rows * 2 * x.shape[1], device=dy.device, dtype=torch.float32)
            dx = K.conv_dgrad_s2_bf16(dy, w, H, W, pd, add=add, part=part, **_bn_kwargs(req))
            back.fill(part, rows, dx)
            return dx
        return K.conv_dgrad_s2_bf16(dy, w, H, W, pd, add=add)
    if w.shape[2] == 1:
        return K.conv_fwd_bf16(dy, w.reshape(w.shape[0], w.shape[1]).t().contiguous(), 1, 1, 0, add=add)
    _, wd = _weight_layouts(w, True)
    return K.conv3x3_fwd_bf16(dy, wd, add=add)


class _ConvGeneralFn(torch.autograd.Function):
    """Strided 3x3 / 1x1 convolution (the downsampling blocks), all three passes on HIP kernels:
    forward and weight gradient on the im2col implicit-GEMM kernels, the input gradient (a transposed
    strided convolution) on the parity-class GEMMs (``_general_dgrad``)."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, part=None, link=None, back=None):
        K = kernels()
        ks = w.shape[2]
        wt = _weight_layouts(w, False)[0] if ks == 3 else w  # [Co][C][1][1] is already [Co][1][C]
        y = K.conv_fwd_bf16(x, wt, ks, stride, pad, part=part)
        ctx.save_for_backward(x)
        ctx.w, ctx.stride, ctx.pad, ctx.link, ctx.back = w, stride, pad, link, back
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, st, pd = ctx.w, ctx.stride, ctx.pad
        dy = dy.contiguous(memory_format=torch.channels_last)
        gw = None
        late = None
        if ctx.needs_input_grad[1]:  # (on the side stream it runs beside the input gradient)
            if w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == torch.bfloat16:
                g = w.grad
                late = _side_wgrad(lambda: kernels().conv_wgrad_bf16_(dy, x, g, st, pd), dy, x, ctx.needs_input_grad[0])
            else:
                gw = torch.zeros_like(w)
                kernels().conv_wgrad_bf16_(dy, x, gw, st, pd)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _general_dgrad(dy, x, w, st, pd, add=_take_addend(ctx.link), back=ctx.back)
        if late is not None:
            late()
        ctx.back = None
        return dx, gw, None, None, None, None, None


def general_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    w = conv.weight
    ks, st, pd = tuple(conv.kernel_size), tuple(conv.stride), tuple(conv.padding)
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and conv.bias is None and w.is_contiguous()
            and ks in ((3, 3), (1, 1)) and pd == ((ks[0] - 1) // 2,) * 2 and st in ((1, 1), (2, 2))
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


class _StemConvFn(torch.autograd.Function):
    """3x3 convolution of a one-channel image (the MNIST stem): streaming kernels, NHWC output."""

    @staticmethod
    def forward(ctx, x, w):
        x = x.contiguous()
        ctx.save_for_backward(x)
        ctx.w = w
        return kernels().conv_c1_fwd_bf16(x, w)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.w
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        if ctx.needs_input_grad[0]:  # the stem's input is data; kept for completeness
            dx = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1)
        gw = None
        if ctx.needs_input_grad[1]:
            if w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == torch.bfloat16:
                kernels().conv_c1_wgrad_bf16_(dy, x, w.grad)
            else:
                gw = torch.zeros_like(w)
                kernels().conv_c1_wgrad_bf16_(dy, x, gw)
        return dx, gw


def stem_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    w = conv.weight
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and conv.in_channels == 1 and conv.bias is None and tuple(conv.kernel_size) == (3, 3)
            and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (1, 1) and tuple(conv.dilation) == (1, 1)
            and conv.groups == 1 and conv.out_channels % 16 == 0 and conv.out_channels <= 512)


# A GPU tensor that no hand-written kernel takes (an fp32 ResNet, an NCHW or odd-width activation) is refused, not
# sent to MIOpen / ATen: on a ROCm device the ResNet runs on conv_bf16.hip / batchnorm_nhwc.hip only, in bf16
# channels-last (fp32 is the CPU / reference-numerics dtype). SDML_CONV_LIBRARY=1 (or LIBRARY_ON_GPU = True) lets
# the A/B tests run the library path as a reference.
LIBRARY_ON_GPU = __import__("os").environ.get("SDML_CONV_LIBRARY", "0") == "1"


def _refuse_library(x: torch.Tensor, what: str):
    if x.is_cuda and not LIBRARY_ON_GPU:
        raise RuntimeError(
            f"{what} on a ROCm device with a {x.dtype} {tuple(x.shape)} activation: no hand-written gfx950 kernel "
            "takes it (the ResNet kernels are bf16 channels-last; run --model resnet18 with --dtype bf16 on the GPU, "
            "fp32 on the CPU). SDML_CONV_LIBRARY=1 allows the MIOpen/ATen path for A/B comparisons.")


def conv2d(conv: torch.nn.Conv2d, x: torch.Tensor, part=None, link=None, back=None) -> torch.Tensor:
    """``conv(x)``, on the HIP kernels where they apply: stride-1 3x3 on the halo kernel, strided
    3x3 / 1x1 on the im2col kernel (input gradient on the parity-class kernel), the streaming stem
    kernels for a one-channel input. ``part`` / ``link`` / ``back``: see ``conv_stats`` / ``ResidualLink`` /
    ``BNBackLink`` (the implicit-GEMM paths only)."""
    if hip_eligible(x, conv):
        return _Conv3x3Fn.apply(x, conv.weight, part, link, back)
    if general_eligible(x, conv):
        return _ConvGeneralFn.apply(x, conv.weight, conv.stride[0], conv.padding[0], part, link, back)
    if stem_eligible(x, conv):
        return _StemConvFn.apply(x, conv.weight)
    _refuse_library(x, "convolution")
    return conv(x)


def conv_stats(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, x: torch.Tensor, link=None, back=None):
    """(y, part): y = conv(x); part = the BatchNorm partials of y written by the convolution's
    epilogue (per 256-pixel tile: channel sums of y and y^2) when the convolution runs on an
    implicit-GEMM kernel and ``bn`` trains on the HIP path, else None. ``batch_norm(bn, y,
    part=part)`` then skips its statistics pass over y."""
    part = None
    if bn.training and (hip_eligible(x, conv) or general_eligible(x, conv)) and bn.weight.dtype == torch.bfloat16:
        N, Co = x.shape[0], conv.out_channels
        OH = (x.shape[2] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
        OW = (x.shape[3] + 2 * conv.padding[1] - conv.kernel_size[1]) // conv.stride[1] + 1
        part = torch.empty(kernels().conv_part_rows(N, OH, OW) * 2 * Co, device=x.device, dtype=torch.float32)
    return conv2d(conv, x, part, link, back), part


# ---- BatchNorm (+ residual) (+ ReLU), channels-last bf16 (csrc/kernels/batchnorm_nhwc.hip) -----
class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, gamma, beta, bn: torch.nn.BatchNorm2d, relu: bool, part=None, back=None):
        momentum = 0.1 if bn.momentum is None else bn.momentum
        nbt = bn.num_batches_tracked  # incremented inside the statistics kernel
        y, mean, rstd = kernels().bn_nhwc_fwd(x, res, gamma, beta, bn.running_mean, bn.running_var, bn.eps,
                                              momentum, relu, nbt if nbt is not None and nbt.is_cuda else None,
                                              part=part)
        if nbt is not None and not nbt.is_cuda:
            nbt.add_(1)
        # BatchNorm + ReLU without a residual: the backward recomputes the mask from x, so y is
        # neither kept alive nor re-read
        keep_y = relu and res is not None
        ctx.save_for_backward(x, y if keep_y else None, mean, rstd)
        ctx.gamma, ctx.beta, ctx.relu, ctx.has_res = gamma, beta, relu, res is not None
        ctx.back = back
        if back is not None:  # detached views: the link must not hold this node's own output (no reference cycle)
            back.args = (x.detach(), y.detach() if keep_y else None, mean, rstd, gamma.detach(), beta.detach(),
                         0 if not relu else (1 if keep_y else 2))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.gamma, ctx.beta
        dy = dy.contiguous(memory_format=torch.channels_last)

        def acc(p):  # the flat-buffer gradient (accumulated in place) or a fresh zero tensor
            if p.grad is not None and p.grad.is_contiguous() and p.grad.dtype == torch.bfloat16:
                return p.grad, False
            return torch.zeros_like(p), True

        gg, own_g = acc(gamma)
        gb, own_b = acc(beta)
        part, rows = ctx.back.take(dy) if ctx.back is not None else (None, 0)
        ctx.back = None
        dx, dres = kernels().bn_nhwc_bwd(x, dy, y if ctx.relu else None, mean, rstd, gamma, ctx.relu, ctx.has_res,
                                          gg, gb, beta, part=part, part_rows=rows)
        return dx, dres, (gg if own_g else None), (gb if own_b else None), None, None, None, None


def bn_eligible(x: torch.Tensor, bn: torch.nn.BatchNorm2d, res=None) -> bool:
    ok = (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and bn.affine and bn.track_running_stats
          and bn.weight.dtype == torch.bfloat16 and x.shape[1] % 8 == 0 and x.shape[1] <= 2048
          and x.is_contiguous(memory_format=torch.channels_last))
    if ok and res is not None:
        ok = res.shape == x.shape and res.dtype == x.dtype and res.is_contiguous(memory_format=torch.channels_last)
    return ok


def batch_norm(bn: torch.nn.BatchNorm2d, x: torch.Tensor, res=None, relu: bool = False, part=None,
               back=None) -> torch.Tensor:
    """``relu?(bn(x) (+ res))`` — one pass per direction on the HIP kernels where they apply; ``part``:
    x's statistics partials from its convolution's epilogue (``conv_stats``); ``back``: a ``BNBackLink`` the
    convolution consuming the output takes, so the backward statistics come from its input-gradient epilogue."""
    if x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4:
        # MIOpen may hand back NCHW (e.g. the 1-channel stem): one copy beats PyTorch's NCHW
        # BatchNorm backward (~0.8 ms per call at batch 512)
        x = x.contiguous(memory_format=torch.channels_last)
        if res is not None:
            res = res.contiguous(memory_format=torch.channels_last)
    if bn_eligible(x, bn, res):
        if bn.training:
            return _BNFn.apply(x, res, bn.weight, bn.bias, bn, relu, part, back)
        with torch.no_grad():
            scale = (bn.weight.float() * torch.rsqrt(bn.running_var.float() + bn.eps)).contiguous()
            shift = (bn.bias.float() - bn.running_mean.float() * scale).contiguous()
        return kernels().bn_nhwc_eval(x, res, scale, shift, relu)
    _refuse_library(x, "BatchNorm")
    y = bn(x)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y
