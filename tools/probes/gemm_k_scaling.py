"""Fixed vs per-K-step cost of the 4-phase bf16 NT GEMM (gemm_bf16.hip) at the GPT-2 tile counts: time at
M = 16384, N = 3072 for K = 768, 1536, 3072, with and without the epilogue's stores (knob GEMM_BF16_NOSTORE,
experiments build: copy exp/_kernels_exp.so over the package .so first), and hipBLASLt alongside."""
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
    return s.elapsed_time(e) / it * 1e3


M, N = 16384, int(os.environ.get("N", 3072))
for Kd in (768, 1536, 3072):
    a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
    row = {"M": M, "N": N, "K": Kd}
    for ns in (0, 1):
        ok = K.set_knob("GEMM_BF16_NOSTORE", ns)
        if not ok and ns:
            continue
        row["hand_nostore" if ns else "hand"] = round(timeit(lambda: K.gemm_bf16(a, w, None, False, 0)), 1)
    K.reset_knobs()
    row["lib"] = round(timeit(lambda: a @ w.t()), 1)
    print(json.dumps(row), flush=True)
