"""Causal flash attention (csrc/kernels/attention.hip) at the GPT-2 bench shape: time forward and
backward, report TF/s (causal FLOPs), and check against PyTorch SDPA in fp32.

    python tools/attn_prof.py [--B 16 --S 1024 --H 12] [--iters 10]
Also the workload for rocprofv3 counter passes (tools/gpu_attn.sh).
"""
import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    K = kernels()
    from simple_distributed_machine_learning_amd._native import apply_knobs_from_env

    knobs = apply_knobs_from_env()  # A/B: SDML_KNOBS="ATTN_DKDV_KT=2", ...
    B, S, H, D = a.B, a.S, a.H, 64
    C = H * D
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(B, S, 3 * C, generator=g).to("cuda", torch.bfloat16)
    q, k, v = (qkv[..., i * C:(i + 1) * C].view(B, S, H, D) for i in range(3))
    dout = torch.randn(B, S, H, D, generator=g).to("cuda", torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    out, lse = K.attention_fwd(q, k, v, scale, True)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = (dqkv[..., i * C:(i + 1) * C].view(B, S, H, D) for i in range(3))
    K.attention_bwd(q, k, v, out, dout, lse, dq, dk, dv, scale, True)
    torch.cuda.synchronize()
    # numerics on one batch element vs fp32 SDPA
    qr, kr, vr = (t[:1].float().transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    yr = F.scaled_dot_product_attention(qr, kr, vr, is_causal=True)
    yr.backward(dout[:1].float().transpose(1, 2))
    err = {n: float((x[:1].float().transpose(1, 2) - r).abs().max() / r.abs().max())
           for n, x, r in (("out", out, yr.detach()), ("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad))}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters * 1e3

    t_f = timed(lambda: K.attention_fwd(q, k, v, scale, True))
    t_b = timed(lambda: K.attention_bwd(q, k, v, out, dout, lse, dq, dk, dv, scale, True))
    fl_f = 4 * B * H * S * S * D / 2  # causal: half of QK^T and PV
    print(json.dumps({"knobs": knobs, "B": B, "S": S, "H": H, "fwd_us": round(t_f, 1), "bwd_us": round(t_b, 1),
                      "fwd_tflops": round(fl_f / t_f / 1e6, 1), "bwd_tflops": round(2.5 * fl_f / t_b / 1e6, 1),
                      "rel_err": {n: round(x, 5) for n, x in err.items()}}), flush=True)


if __name__ == "__main__":
    main()
