"""Accuracy/speed probe of the bf16x3 fp32 GEMM engine pipeline variants (0: split of tile t+1
interleaved with tile t's MFMAs, 1: split after the MFMAs) against the exact fp32-input MFMA
engine and fp64.

    python tools/x3_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native, ops  # noqa: E402

K = _native.kernels()
dev = torch.device("cuda", 0)


def rnd(*s, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.empty(s).uniform_(lo, hi, generator=g).to(dev)


def timeit(fn, iters=20):
    for _ in range(5):
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
    return sorted(ts)[len(ts) // 2]


for Kd in (784, 4096):
    A, B = rnd(512, Kd, seed=3), rnd(256, Kd, seed=4)
    want = A.double() @ B.double().t()
    C = torch.empty(512, 256, device=dev)
    K.gemm_f32_set_mode(0)
    K.gemm_f32(A, B, C, False, False, 0)
    e = (C.double() - want).abs()
    print(f"K={Kd} fp32-mfma  max {e.max():.3e} mean {e.mean():.3e}")
    for v in (0, 1):
        K.gemm_f32x3_set_variant(v)
        K.gemm_f32x3(A, B, C, False, False, 0)
        e = (C.double() - want).abs()
        print(f"K={Kd} x3 var{v}   max {e.max():.3e} mean {e.mean():.3e} bias {(C.double() - want).mean():.3e}")
K.gemm_f32_set_mode(1)
Bt, Kd, N = 131072, 784, 128
x, w, b = rnd(Bt, Kd, seed=1, lo=0, hi=1), rnd(N, Kd, seed=2) * 0.05, rnd(N, seed=3) * 0.1
h = ops.linear_relu_fwd(x, w, b)
gy = rnd(Bt, N, seed=4) * 1e-3 * (h > 0)
gw, gb = torch.zeros_like(w), torch.zeros_like(b)
fl = 2.0 * Bt * Kd * N
variants = [int(v) for v in os.environ.get("X3_VARIANTS", "0,1").split(",")]
outs = {}
for v in variants:
    K.gemm_f32x3_set_variant(v)
    outs[v] = ops.linear_relu_fwd(x, w, b)
for v in variants[1:]:
    print(f"variant {v} fwd vs variant {variants[0]}: max |diff| {(outs[v] - outs[variants[0]]).abs().max():.3e}")
for v in variants + variants:
    K.gemm_f32x3_set_variant(v)
    tf = timeit(lambda: ops.linear_relu_fwd(x, w, b))
    tw = timeit(lambda: ops.linear_relu_bwd(x, h, gy, w, gw, gb, False, gy_masked=True))
    print(f"variant {v}: fwd {tf*1e3:.1f} us ({fl/tf/1e9:.1f} TF/s)  dW {tw*1e3:.1f} us ({fl/tw/1e9:.1f} TF/s)")
K.gemm_f32x3_set_variant(0)
