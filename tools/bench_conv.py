"""Per-call time of the ResNet convolution kernels at the bf16 ResNet-18 (batch 512, 28x28 MNIST)
shapes, with and without the fused epilogue operands (BatchNorm partials, residual addend).

    python tools/bench_conv.py            -> one JSON line per (kernel, shape, epilogue)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
DEV = torch.device("cuda", 0)


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    N = int(os.environ.get("BATCH", "512"))
    for C, Co, H in [(64, 64, 28), (128, 128, 14), (256, 256, 7), (512, 512, 4)]:
        x = cl(torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16))
        w = (torch.randn(Co, C, 3, 3, device=DEV) * 0.05).to(torch.bfloat16)
        wt = K.conv3x3_weight_bf16(w, False)
        add = cl(torch.randn(N, Co, H, H, device=DEV).to(torch.bfloat16))
        part = torch.empty(K.conv_part_rows(N, H, H) * 2 * Co, device=DEV)
        flops = 2 * N * H * H * Co * C * 9
        for name, fn in [("plain", lambda: K.conv3x3_fwd_bf16(x, wt)),
                         ("part", lambda: K.conv3x3_fwd_bf16(x, wt, part=part)),
                         ("add", lambda: K.conv3x3_fwd_bf16(x, wt, add=add))]:
            us = timed(fn)
            print(json.dumps({"kernel": "conv3x3_s1", "C": C, "Co": Co, "H": H, "epi": name, "us": round(us, 2),
                              "tflops": round(flops / us / 1e6, 1)}))
    for C, Co, H in [(64, 128, 28), (128, 256, 14), (256, 512, 7)]:
        OH = (H + 1) // 2
        dy = cl(torch.randn(N, Co, OH, OH, device=DEV).to(torch.bfloat16))
        add = cl(torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16))
        for ks, pd in [(3, 1), (1, 0)]:
            w = (torch.randn(Co, C, ks, ks, device=DEV) * 0.05).to(torch.bfloat16)
            flops = 2 * N * OH * OH * Co * C * ks * ks
            for name, fn in [("plain", lambda: K.conv_dgrad_s2_bf16(dy, w, H, H, pd)),
                             ("add", lambda: K.conv_dgrad_s2_bf16(dy, w, H, H, pd, add=add))]:
                us = timed(fn)
                print(json.dumps({"kernel": f"dgrad_s2_{ks}x{ks}", "C": C, "Co": Co, "H": H, "epi": name,
                                  "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}))


if __name__ == "__main__":
    main()
