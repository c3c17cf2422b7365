"""ResNet-18-style CNN on MNIST-shape input, split into up to 8 pipeline stages
(BASELINE config 4: "8-stage ResNet-18-style CNN across 8 MI355X with 1F1B").

Architecture (CIFAR-style stem for 28x28 inputs): conv3x3(1->64)+BN+ReLU, then 4 layers of
2 BasicBlocks (64, 128/2, 256/2, 512/2), global average pool, fc(512->10).
The 8 BasicBlocks are the cut units: stage k gets ``8 / num_stages`` consecutive blocks;
the stem rides with the first stage and pool+fc with the last.

BatchNorm runs per micro-batch (GPipe semantics). ``dtype=bf16`` (the GPU default of the benchmarks)
runs the stages in bf16 channels-last (fp32 master weights in the optimizer) on hand-written kernels
only: every convolution in csrc/kernels/conv_bf16.hip — the stride-1 3x3 convolutions (forward, input
and weight gradients), the stride-2 3x3 and 1x1 shortcut convolutions (forward, weight gradient, and the
input gradient as parity-class GEMMs), the one-channel stem — every BatchNorm(+residual)(+ReLU) in
csrc/kernels/batchnorm_nhwc.hip, and the last stage's average pool + fc + log_softmax + NLL + backward
in csrc/kernels/head_pool.hip. ``dtype=fp32`` is the CPU / reference-numerics path; on a GPU it is refused
(ops/conv.py ``_refuse_library``: no MIOpen / ATen convolution on the device), and ``train.py`` picks bf16 for
``--model resnet18`` on a GPU unless ``--dtype`` says otherwise.
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import ModelSpec, PipelineStage
from .. import ops
from ..ops import conv as conv_ops

WIDTHS = (64, 128, 256, 512)
# fp32 runs NCHW on MIOpen (channels-last fp32 measured slower there); bf16 runs channels-last so
# the stride-1 3x3 convolutions take the hand-written implicit-GEMM kernels (ops/conv.py)
CHANNELS_LAST = os.environ.get("SDML_RESNET_NHWC", "auto")


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x, back=None):
        return self.forward_linked(x, back)[0]

    def forward_linked(self, x, back=None):
        """(out, link). conv (HIP implicit GEMM when bf16 NHWC; the epilogue also writes the BatchNorm statistics
        partials) -> BN+ReLU / BN+residual+ReLU in one pass each (ops/conv.py; PyTorch ops elsewhere).
        The residual branch's input gradient is added in conv1's input-gradient epilogue (ResidualLink): the tap
        on x is created after the main branch's convolutions so autograd runs it first. BatchNorm backward
        statistics come from the input-gradient epilogue of the convolution consuming the BatchNorm's output
        (BNBackLink): bn1's from conv2's, and ``back`` (the BatchNorm that produced x) from conv1's when the
        residual gradient was fused there; ``link`` is bn2's, for the next block's conv1."""
        gpu_bf16 = x.is_cuda and x.dtype == torch.bfloat16
        link = conv_ops.ResidualLink() if (conv_ops.FUSE_RESIDUAL and x.requires_grad and gpu_bf16) else None
        fuse = conv_ops.FUSE_BN_BACK and gpu_bf16 and torch.is_grad_enabled() and self.training
        b1 = conv_ops.BNBackLink() if fuse else None
        b2 = conv_ops.BNBackLink(needs_addend=True) if fuse else None
        y1, p1 = conv_ops.conv_stats(self.conv1, self.bn1, x, link, back=back)
        out = conv_ops.batch_norm(self.bn1, y1, relu=True, part=p1, back=b1)
        if self.shortcut is None:
            y2, p2 = conv_ops.conv_stats(self.conv2, self.bn2, out, back=b1)
            sc = conv_ops.grad_tap(x, link)
        else:
            ys, ps = conv_ops.conv_stats(self.shortcut[0], self.shortcut[1], conv_ops.grad_tap(x, link))
            sc = conv_ops.batch_norm(self.shortcut[1], ys, part=ps)
            y2, p2 = conv_ops.conv_stats(self.conv2, self.bn2, out, back=b1)
        return conv_ops.batch_norm(self.bn2, y2, res=sc, relu=True, part=p2, back=b2), b2


def block_defs(in_ch: int = 1):
    defs = []
    cin = 64
    for li, w in enumerate(WIDTHS):
        for bi in range(2):
            stride = 2 if (li > 0 and bi == 0) else 1
            defs.append((f"layer{li + 1}.{bi}", cin, w, stride))
            cin = w
    return defs


def _nhwc(dtype) -> bool:
    return CHANNELS_LAST == "1" or (CHANNELS_LAST == "auto" and dtype == torch.bfloat16)


class ResNetStage(PipelineStage):
    def __init__(self, stage_id: int, num_stages: int, in_ch: int = 1, num_classes: int = 10,
                 boundary_nhwc: bool = False):
        super().__init__()
        # channels-last runs hand the boundary tensor over as a contiguous [N, H, W, C] array (the
        # same bytes as the channels-last activation): no NCHW <-> NHWC copy at each stage cut
        self.boundary_nhwc = boundary_nhwc
        if 8 % num_stages:
            raise ValueError("resnet18 splits into 1, 2, 4 or 8 stages")
        self.stage_id, self.num_stages = stage_id, num_stages
        per = 8 // num_stages
        defs = block_defs(in_ch)[stage_id * per:(stage_id + 1) * per]
        self.loss_kind = "ce"
        if stage_id == 0:
            self.stem_conv = nn.Conv2d(in_ch, 64, 3, 1, 1, bias=False)
            self.stem_bn = nn.BatchNorm2d(64)
        self.block_names = []
        for name, cin, cout, stride in defs:
            attr = name.replace(".", "_")
            setattr(self, attr, BasicBlock(cin, cout, stride))
            self.block_names.append(attr)
        if stage_id == num_stages - 1:
            self.fc = nn.Linear(512, num_classes)

    def trunk(self, x):
        """Everything but the last stage's pool + fc.
        NHWC inside the stage for bf16 (SDML_RESNET_NHWC=auto; 1/0 force it on/off). Measured on
        MI355X (8 stages on one GPU, batch 512, 8 micro-batches): MIOpen picks slower solutions
        for channels-last fp32 (9.6K vs 14.6K samples/s), so fp32 stays NCHW. The boundary
        tensor is NCHW, or [N, H, W, C] in channels-last runs (boundary_nhwc)."""
        if self.stage_id == 0:
            x = x.to(self.stem_conv.weight.dtype)
        elif self.boundary_nhwc:
            x = x.permute(0, 3, 1, 2)  # [N, H, W, C] boundary -> channels-last NCHW view, no copy
        nhwc = _nhwc(x.dtype)
        if x.is_cuda and nhwc:
            x = x.contiguous(memory_format=torch.channels_last)
        back = None  # BNBackLink of the BatchNorm that produced x (BasicBlock.forward_linked)
        if self.stage_id == 0:
            if conv_ops.FUSE_BN_BACK and x.is_cuda and nhwc and torch.is_grad_enabled() and self.training:
                back = conv_ops.BNBackLink(needs_addend=True)
            x = conv_ops.batch_norm(self.stem_bn, conv_ops.conv2d(self.stem_conv, x), relu=True, back=back)
        for n in self.block_names:
            x, back = getattr(self, n).forward_linked(x, back)
        return x

    def forward(self, x):
        x = self.trunk(x)
        if self.stage_id == self.num_stages - 1:
            x = F.adaptive_avg_pool2d(x, 1).flatten(1)
            x = self.fc(x)
            return x
        if self.boundary_nhwc:
            return x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        return x.contiguous()

    # Training head on ROCm: pool + fc + log_softmax + NLL + backward in one kernel (+ its reduction),
    # ops.pooled_head_xent / head_pool.hip, instead of ATen pooling, a hipBLASLt GEMM and ATen
    # log_softmax / nll_loss forward and backward (the reference's loss: simple_distributed.py:111).
    # SDML_RESNET_HEAD=aten keeps the autograd head.
    def head_fwd(self, x, target, ctx, train, loss_scale, stats=None):
        fc = getattr(self, "fc", None)
        if not (train and x.is_cuda and fc is not None and stats is not None and fc.weight.grad is not None
                and os.environ.get("SDML_RESNET_HEAD", "fused") != "aten"):
            return super().head_fwd(x, target, ctx, train, loss_scale, stats)
        if not self.is_first:
            x = x.detach().requires_grad_(True)
        with torch.enable_grad():
            y = self.trunk(x)
            if not ops.pooled_head_ok(y, fc.weight):
                # finish the autograd head on this y (the trunk - and its BatchNorm running-stat updates - ran
                # once; re-running the whole forward through super().head_fwd would run them twice)
                out = fc(F.adaptive_avg_pool2d(y, 1).flatten(1))
                loss, correct, n = self.loss_terms(out, target)
                ctx["x"], ctx["loss"] = x, loss * loss_scale
                return loss.detach(), correct.detach(), n
        ctx["x"], ctx["y"] = x, y
        ctx["gy"] = ops.pooled_head_xent(y.detach(), fc.weight, fc.bias, target, fc.weight.grad, fc.bias.grad,
                                         loss_scale, stats)
        return None, None, target.numel()

    def head_bwd(self, ctx):
        if "gy" not in ctx:
            return super().head_bwd(ctx)
        y, gy, x = ctx.pop("y"), ctx.pop("gy"), ctx.pop("x")
        torch.autograd.backward(y, gy)
        return None if self.is_first else x.grad


def _out_shape(stage: int, num_stages: int, hw: int = 28):
    per = 8 // num_stages
    last_block = (stage + 1) * per - 1
    defs = block_defs()
    c = defs[last_block][2]
    size = hw
    for i in range(last_block + 1):
        if defs[i][3] == 2:
            size = (size + 1) // 2
    return c, size


def resnet18_spec(num_stages: int = 8, dtype=torch.float32) -> ModelSpec:
    nhwc = _nhwc(dtype) and torch.cuda.is_available()

    def build(s):
        return ResNetStage(s, num_stages, boundary_nhwc=nhwc)

    def shape(s, mb):
        c, hw = _out_shape(s, num_stages)
        return (mb, hw, hw, c) if nhwc else (mb, c, hw, hw)

    return ModelSpec(name="resnet18", num_stages=num_stages, build_stage=build, boundary_shape=shape,
                     boundary_dtype=dtype, input_kind="image", param_dtype=dtype)
