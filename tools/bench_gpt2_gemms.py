"""Per-shape timing of the GPT-2-small projection GEMMs (bf16, hipBLASLt through torch) at
the single-GPU step shape (16 x 1024 tokens), with weight-gradient variants.

    python tools/bench_gpt2_gemms.py [--tokens 16384]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--tuned", action="store_true")
    a = ap.parse_args()
    if a.tuned:
        from simple_distributed_machine_learning_amd.utils.tuned_gemm import use_tuned_gemms
        print("tuned:", use_tuned_gemms())
    dev = torch.device("cuda", 0)
    from simple_distributed_machine_learning_amd import _native
    K = _native.kernels()
    T = a.tokens
    bf = torch.bfloat16
    for (inf, outf) in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        x = torch.randn(T, inf, device=dev, dtype=bf)
        w = torch.randn(outf, inf, device=dev, dtype=bf) * 0.02
        b = torch.zeros(outf, device=dev, dtype=bf)
        gy = torch.randn(T, outf, device=dev, dtype=bf)
        gw = torch.zeros(outf, inf, device=dev, dtype=bf)
        fl = 2.0 * T * inf * outf
        res = {}
        res["fwd addmm"] = timeit(lambda: torch.addmm(b, x, w.t()))
        res["dX gy@w"] = timeit(lambda: gy @ w)
        res["dW addmm_"] = timeit(lambda: gw.addmm_(gy.t(), x))
        res["dW mm fp32out"] = timeit(lambda: torch.mm(gy.t(), x, out_dtype=torch.float32))
        res["dW wgrad_bf16 (HIP)"] = timeit(lambda: K.wgrad_bf16_(gy, x, gw))
        gb = torch.zeros(outf, device=dev, dtype=bf)
        res["dW+db wgrad_bf16 (HIP)"] = timeit(lambda: K.wgrad_bf16_(gy, x, gw, gb))
        for S in (8,):
            gs = gy.view(S, T // S, outf).transpose(1, 2)
            xs = x.view(S, T // S, inf)
            res[f"dW bmm S={S} fp32 + sum"] = timeit(
                lambda: gw.add_(torch.bmm(gs, xs, out_dtype=torch.float32).sum(0)))
        print(f"[{inf}->{outf}] " + "  ".join(f"{k}: {v:.1f}us ({fl / v / 1e6:.0f} TF/s)" for k, v in res.items()),
              flush=True)
    # lm_head
    x = torch.randn(T, 768, device=dev, dtype=bf)
    w = torch.randn(50257, 768, device=dev, dtype=bf) * 0.02
    gy = torch.randn(T, 50257, device=dev, dtype=bf)
    gw = torch.zeros_like(w)
    fl = 2.0 * T * 768 * 50257
    print("[lm_head] fwd %.1f us, dX %.1f us, dW %.1f us (flops/GEMM %.2f T)" % (
        timeit(lambda: x @ w.t(), 5), timeit(lambda: gy @ w, 5), timeit(lambda: gw.addmm_(gy.t(), x), 5), fl / 1e12))


if __name__ == "__main__":
    main()
