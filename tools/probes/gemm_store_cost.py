"""Timing probe (experiments build: knob GEMM_BF16_NOSTORE): what the epilogue's HBM stores cost the bf16 NT GEMM at
the GPT-2 shapes, per epilogue (bias; bias + GELU saving gelu'), with and without the stores."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
dev = torch.device("cuda", 0)


def timeit(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / it * 1e3, 1)


T = 16384
for name, N, Kd, epis in (("c_attn", 2304, 768, (1,)), ("attn.c_proj", 768, 768, (1,)), ("c_fc", 3072, 768, (1, 7)),
                          ("mlp.c_proj", 768, 3072, (1,)), ("lm_head", 50304, 768, (0,))):
    x = torch.randn(T, Kd, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    aux = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    r = {"gemm": name, "M": T, "N": N, "K": Kd}
    for epi in epis:
        for ns in (0, 1):
            K.set_knob("GEMM_BF16_NOSTORE", ns)
            fn = (lambda: K.gemm_bf16(x, w, b, False, epi, aux)) if epi == 7 else (lambda: K.gemm_bf16(x, w, b if epi else None, False, epi))
            r[f"epi{epi}_us" + ("_nostore" if ns else "")] = timeit(fn)
        K.set_knob("GEMM_BF16_NOSTORE", 0)
        out_bytes = T * N * 2 * (2 if epi == 7 else 1)
        r[f"epi{epi}_store_MB"] = round(out_bytes / 1e6, 1)
    print(json.dumps(r), flush=True)
K.reset_knobs()
