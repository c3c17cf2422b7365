"""Minimal driver for rocprofv3 counter passes: 5 x (fwd, dW) of the headline MLP layer on the
bf16x3 engine (variant from argv[1], default 0)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native, ops  # noqa: E402

K = _native.kernels()
K.gemm_f32x3_set_variant(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
Bt, Kd, N = 131072, 784, 128
x = torch.rand(Bt, Kd, device=dev, generator=g)
w = torch.randn(N, Kd, device=dev, generator=g) * 0.05
b = torch.randn(N, device=dev, generator=g) * 0.1
h = ops.linear_relu_fwd(x, w, b)
gy = torch.randn(Bt, N, device=dev, generator=g) * 1e-3 * (h > 0)
gw, gb = torch.zeros_like(w), torch.zeros_like(b)
for _ in range(5):
    ops.linear_relu_fwd(x, w, b)
    ops.linear_relu_bwd(x, h, gy, w, gw, gb, False, gy_masked=True)
torch.cuda.synchronize()
