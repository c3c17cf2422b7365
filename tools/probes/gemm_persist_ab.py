"""A/B (knob GEMM_BF16_PERSIST): the bf16 NT GEMM, one workgroup per tile vs persistent workgroups, at the GPT-2
shapes per epilogue (0 plain, 1 bias, 7 bias + GELU saving gelu', 8 times the saved gelu'), interleaved reps."""
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
shapes = (("c_attn", 2304, 768, (1,)), ("attn.c_proj", 768, 768, (1,)), ("c_fc", 3072, 768, (7,)),
          ("mlp.c_proj", 768, 3072, (1,)), ("c_fc.dx", 768, 3072, (0,)), ("mlp.c_proj.dx", 3072, 768, (8,)),
          ("c_attn.dx", 768, 2304, (0,)), ("lm_head", 50304, 768, (0,)), ("lm_head.dx", 768, 50304, (0,)))
for rep in range(2):
    for name, N, Kd, epis in shapes:
        x = torch.randn(T, Kd, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        aux = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        for epi in epis:
            r = {"gemm": name, "M": T, "N": N, "K": Kd, "epi": epi, "rep": rep}
            for pers in (0, 1):
                K.set_knob("GEMM_BF16_PERSIST", pers)
                if epi in (1, 7):
                    fn = lambda: K.gemm_bf16(x, w, b, False, epi)
                elif epi == 8:
                    fn = lambda: K.gemm_bf16(x, w, None, False, epi, aux)
                else:
                    fn = lambda: K.gemm_bf16(x, w, None, False, epi)
                r[f"persist{pers}_us"] = timeit(fn)
            K.reset_knobs()
            print(json.dumps(r), flush=True)
        del x, w, b, aux
