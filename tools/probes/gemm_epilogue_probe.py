"""Timing probe: gemm_bf16 NT forward at the GPT-2 shapes with and without the epilogue's HBM stores
(SDML_GEMM_BF16_NOSTORE=1), for the plain and the bias+GELU epilogue; hipBLASLt for reference."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
dev = torch.device("cuda", 0)


def timeit(fn, it=20):
    for _ in range(3):
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
for name, N, Kd in (("c_attn", 2304, 768), ("c_fc", 3072, 768), ("mlp.c_proj", 768, 3072)):
    x = torch.randn(T, Kd, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    r = {"gemm": name}
    for ns in ("0", "1"):
        os.environ["SDML_GEMM_BF16_NOSTORE"] = ns
        r["bias_us" + ("_nostore" if ns == "1" else "")] = timeit(lambda: K.gemm_bf16(x, w, b, False, 1))
        r["gelu_us" + ("_nostore" if ns == "1" else "")] = timeit(lambda: K.gemm_bf16(x, w, b, False, 5))
    os.environ["SDML_GEMM_BF16_NOSTORE"] = "0"
    r["hipblaslt_us"] = timeit(lambda: torch.addmm(b, x, w.t()))
    print(json.dumps(r), flush=True)
