"""Micro-benchmark of the MLP hot kernels at bench shapes vs PyTorch/hipBLASLt (fp32).

    python tools/bench_kernels.py [--batch 131072]
Prints one line per kernel: time (median of N, HIP events), achieved TFLOP/s or GB/s.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native, ops  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, K, N, C = a.batch, 784, 128, 10
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, K, device=dev, generator=g)
    w = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g) * 0.1
    h = ops.linear_relu_fwd(x, w, b)
    gy = torch.randn(B, N, device=dev, generator=g) * 1e-3
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    w2, b2 = torch.randn(C, N, device=dev, generator=g) * 0.1, torch.zeros(C, device=dev)
    gw2, gb2 = torch.zeros_like(w2), torch.zeros_like(b2)
    t = torch.randint(0, C, (B,), device=dev, generator=g)
    stats = torch.zeros(2, device=dev)
    fl = 2.0 * B * K * N
    res = {}

    def rep(name, sec, flops=None, bytes_=None):
        d = {"ms": round(sec * 1e3, 4)}
        if flops:
            d["TFLOPs"] = round(flops / sec / 1e12, 1)
        if bytes_:
            d["GBs"] = round(bytes_ / sec / 1e9, 1)
        res[name] = d
        print(name, d, flush=True)

    rep("fwd_gemm_bias_relu", timeit(lambda: ops.linear_relu_fwd(x, w, b)), fl)
    rep("torch_fwd (hipBLASLt addmm+relu)", timeit(lambda: torch.relu(torch.addmm(b, x, w.t()))), fl)
    rep("dW_gemm_masked_rowsum", timeit(lambda: ops.linear_relu_bwd(x, h, gy, w, gw, gb, False)), fl)
    rep("torch_dW (hipBLASLt)", timeit(lambda: torch.mm((gy * (h > 0)).t(), x)), fl)
    rep("dX_gemm_masked", timeit(lambda: ops.linear_relu_bwd(x, h, gy, w, None, None, True)), fl)
    rep("head_fused_fwd_bwd", timeit(lambda: ops.linear_logsoftmax_nll(h, w2, b2, t, gw2, gb2, 1.0 / B, True, stats)),
        bytes_=B * N * 4 * 2 + B * 8)
    # A/B of the two fp32 GEMM engines (bf16x3 split vs exact fp32-input MFMA), interleaved
    # rounds in one process (guide §5.4 rule 24)
    K_ = _native.kernels()
    ab = {1: {"fwd": [], "dW": [], "dX": []}, 0: {"fwd": [], "dW": [], "dX": []}}
    for _ in range(5):
        for v in (1, 0):
            K_.gemm_f32_set_mode(v)
            ab[v]["fwd"].append(timeit(lambda: ops.linear_relu_fwd(x, w, b), iters=10))
            ab[v]["dW"].append(timeit(lambda: ops.linear_relu_bwd(x, h, gy, w, gw, gb, False), iters=10))
            ab[v]["dX"].append(timeit(lambda: ops.linear_relu_bwd(x, h, gy, w, None, None, True), iters=10))
    K_.gemm_f32_set_mode(1)
    for v in ab:
        for k in ab[v]:
            t_ = sorted(ab[v][k])
            rep(f"engine {'bf16x3' if v else 'fp32-mfma'} {k} (median of 5 rounds)", t_[2], fl,
                bytes_=B * K * 4 + B * N * 4)
    p = torch.zeros(101888, device=dev)
    gg, mb = torch.randn_like(p), torch.zeros_like(p)
    rep("sgd", timeit(lambda: ops.sgd_momentum_(p, gg, mb, 0.1, 0.5)), bytes_=p.numel() * 4 * 5)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
