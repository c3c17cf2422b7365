"""Two-fp16-plane fp32 GEMM engine (gemm_f16x2.hip) vs the bf16x3 engine (gemm_f32x3.hip) at the 4x1024
MLP's hidden-layer shapes (65536 x 1024 x 1024 by default): forward (NT, bias + ReLU), input gradient
(NN, ReLU mask), weight + bias gradient, and the split pass. One JSON line.

    python tools/bench_x2.py [--M 65536 --N 1024 --K 1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=1024)
    a = ap.parse_args()
    M, N, Kd = a.M, a.N, a.K
    K = kernels()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(M, Kd, device=dev, generator=g)
    w = torch.rand(N, Kd, device=dev, generator=g) - 0.5
    b = torch.rand(N, device=dev, generator=g)
    dz = torch.rand(M, N, device=dev, generator=g) - 0.5
    gw = torch.zeros(N, Kd, device=dev)
    gb = torch.zeros(N, device=dev)
    inf = lambda t: torch.linalg.vector_norm(t, float("inf")).reshape(1)  # noqa: E731
    px, sx = K.x2_split(x, inf(x))
    pw, sw = K.x2_split(w, inf(w))
    pd, sd = K.x2_split(dz, inf(dz))
    # W as [K][N] for the input gradient's NN layout (the engine stores W [N][K] = [out][in]; dx = dz @ W)
    flops = 2.0 * M * N * Kd
    r = {"shape": [M, N, Kd]}
    r["split_us"] = round(timeit(lambda: K.x2_split(x, inf(x))), 1)
    r["x2_fwd_us"] = round(timeit(lambda: K.x2_gemm(px, sx, pw, sw, False, b, True)), 1)
    r["x2_dx_us"] = round(timeit(lambda: K.x2_gemm(pd, sd, pw, sw, True, None, False, x, True)), 1)
    pwt, swt = K.x2_split_t(w, inf(w))
    r["x2_dx_nt_us"] = round(timeit(lambda: K.x2_gemm(pd, sd, pwt, swt, False, None, False, x, True)), 1)
    r["split_only_us"] = round(timeit(lambda: K.x2_split(x, sx)), 1)
    r["infnorm_us"] = round(timeit(lambda: inf(x)), 1)
    r["x2_wgrad_us"] = round(timeit(lambda: K.x2_wgrad_(pd, sd, px, sx, gw, gb)), 1)
    C = torch.empty(M, N, device=dev)
    r["x3_fwd_us"] = round(timeit(lambda: K.gemm_f32x3(x, w, C, False, False, 2, b)), 1)
    dx = torch.empty(M, Kd, device=dev)
    r["x3_dx_us"] = round(timeit(lambda: K.gemm_f32x3(dz, w, dx, False, True, 0, None, None, None, x)), 1)
    for k in ("x2_fwd", "x2_dx", "x2_dx_nt", "x2_wgrad", "x3_fwd", "x3_dx"):
        r[k + "_fp32_TFs"] = round(flops / r[k + "_us"] / 1e6, 1)
    print(json.dumps(r))


if __name__ == "__main__":
    main()
