"""Flash-attention kernel micro-benchmark (GPT-2 shape by default): HIP kernels vs PyTorch SDPA.

    python tools/bench_attention.py [--B 4 --H 12 --S 1024]
Prints per-pass time and TFLOP/s (causal FLOPs: fwd 2 GEMMs, bwd 5 GEMMs over half the square).
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402


def timeit(fn, iters=50, warm=5):
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
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--fwd_kb", type=int, default=0, help="forward keys per tile (0 = default)")
    a = ap.parse_args()
    B, H, S, D = a.B, a.H, a.S, 64
    dev = torch.device("cuda", 0)
    K = kernels()
    qkv = torch.randn(B, S, 3 * H * D, device=dev, dtype=torch.bfloat16)
    q, k, v = (qkv[..., i * H * D:(i + 1) * H * D].view(B, S, H, D) for i in range(3))
    scale = 1.0 / D ** 0.5
    K.attention_set_fwd_kb(0)
    ref_out, ref_lse = K.attention_fwd(q, k, v, scale, True)
    K.attention_set_fwd_kb(a.fwd_kb)
    out, lse = K.attention_fwd(q, k, v, scale, True)
    err = float((out.float() - ref_out.float()).abs().max())
    dout = torch.randn_like(out)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = (dqkv[..., i * H * D:(i + 1) * H * D].view(B, S, H, D) for i in range(3))
    flops_f = 4.0 * B * H * S * S * D / 2
    flops_b = 10.0 * B * H * S * S * D / 2
    t_f = timeit(lambda: K.attention_fwd(q, k, v, scale, True))
    t_b = timeit(lambda: K.attention_bwd(q, k, v, out, dout, lse, dq, dk, dv, scale, True))
    qt, kt, vt = (x.transpose(1, 2).contiguous().requires_grad_(True) for x in (q, k, v))
    t_sf = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True))
    y = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
    g = torch.randn_like(y)
    t_sb = timeit(lambda: torch.autograd.grad(y, (qt, kt, vt), g, retain_graph=True))
    print(json.dumps({"shape": [B, H, S, D], "fwd_kb": a.fwd_kb, "max_diff_vs_default": err, "hip_fwd_us": round(t_f, 1), "hip_fwd_tflops": round(flops_f / t_f / 1e6, 1),
                      "hip_bwd_us": round(t_b, 1), "hip_bwd_tflops": round(flops_b / t_b / 1e6, 1),
                      "sdpa_fwd_us": round(t_sf, 1), "sdpa_bwd_us": round(t_sb, 1)}))


if __name__ == "__main__":
    main()
