"""Per-layer timing of the ResNet-18 stride-1 3x3 convolutions (batch 512, MNIST-shape stages) on the
hand-written kernels (csrc/kernels/conv_bf16.hip) next to MIOpen, with a numerics check of each
kernel against F.conv2d (fp32 accumulate of the same bf16 operands).

    python tools/bench_conv.py [--batch 512] [--iters 20]
    SDML_CONV_FWD=im2col python tools/bench_conv.py     # A/B the forward kernel variants
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402

LAYERS = [(28, 64), (14, 128), (7, 256), (4, 512)]  # (H = W, channels) of layer1..layer4


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    K = kernels()
    g = torch.Generator(device="cpu").manual_seed(0)
    cl = torch.channels_last
    for hw, c in LAYERS:
        N = a.batch
        x = torch.randn(N, c, hw, hw, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(N, c, hw, hw, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(c, c, 3, 3, generator=g) * (2.0 / (9 * c)) ** 0.5).to("cuda", torch.bfloat16)
        wt, wd = K.conv3x3_weight_bf16(w, False), K.conv3x3_weight_bf16(w, True)
        gw = torch.zeros_like(w)
        flops = 2 * N * hw * hw * c * c * 9
        y = K.conv3x3_fwd_bf16(x, wt)
        yr = F.conv2d(x.float(), w.float(), padding=1)
        err_f = float((y.float() - yr).abs().max() / yr.abs().max())
        dx = K.conv3x3_fwd_bf16(dy, wd)
        dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), padding=1)
        err_d = float((dx.float() - dxr).abs().max() / dxr.abs().max())
        gw.zero_()
        K.conv3x3_wgrad_bf16_(dy, x, gw)
        gwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), padding=1)
        err_w = float((gw.float() - gwr).abs().max() / gwr.abs().max())
        t_f = timed(lambda: K.conv3x3_fwd_bf16(x, wt), a.iters)
        t_d = timed(lambda: K.conv3x3_fwd_bf16(dy, wd), a.iters)
        t_w = timed(lambda: K.conv3x3_wgrad_bf16_(dy, x, gw), a.iters)
        t_mf = timed(lambda: F.conv2d(x, w, padding=1), a.iters)
        print(json.dumps({"hw": hw, "c": c, "fwd_us": round(t_f, 1), "dgrad_us": round(t_d, 1),
                          "wgrad_us": round(t_w, 1), "fwd_tflops": round(flops / t_f / 1e6, 1),
                          "wgrad_tflops": round(flops / t_w / 1e6, 1), "miopen_fwd_us": round(t_mf, 1),
                          "rel_err": [round(err_f, 5), round(err_d, 5), round(err_w, 5)],
                          "engine": os.environ.get("SDML_CONV_FWD", "halo")}), flush=True)


if __name__ == "__main__":
    main()
