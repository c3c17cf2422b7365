"""gemm_bf16.hip against torch.matmul (hipBLASLt) on the GPT-2 small shapes (T = 16384 tokens):
forward (NT, X W^T) and input gradient (NN, dY W) of c_attn, attn.c_proj, mlp.c_fc, mlp.c_proj and
the (vocab-padded) lm_head. Checks each result against an fp32 matmul and prints TF/s of both."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
_native.apply_knobs_from_env()  # e.g. SDML_KNOBS=GEMM_BF16_T2=1 (the 256 x 128, two-workgroups-per-CU NT kernel)
dev = torch.device("cuda", 0)
T = int(os.environ.get("T", 16384))
SHAPES = [("c_attn", 2304, 768), ("attn.c_proj", 768, 768), ("c_fc", 3072, 768), ("mlp.c_proj", 768, 3072),
          ("lm_head", 50304, 768)]


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
    return s.elapsed_time(e) / it * 1e3  # us


g = torch.Generator(device="cpu").manual_seed(0)
for name, N, Kd in SHAPES:
    w = (torch.randn(N, Kd, generator=g) * 0.02).to(dev, torch.bfloat16)
    b = (torch.randn(N, generator=g) * 0.02).to(dev, torch.bfloat16)
    x = torch.randn(T, Kd, generator=g).to(dev, torch.bfloat16)
    gy = torch.randn(T, N, generator=g).to(dev, torch.bfloat16)
    flops = 2.0 * T * N * Kd
    # forward
    y, _ = K.gemm_bf16(x, w, b, False, 1)
    ref = x.float() @ w.float().t() + b.float()
    err_f = float((y.float() - ref).abs().max() / ref.abs().max())
    t_mine = timeit(lambda: K.gemm_bf16(x, w, b, False, 1))
    t_lib = timeit(lambda: torch.addmm(b, x, w.t()))
    # input gradient
    dx, _ = K.gemm_bf16(gy, w, None, True, 0)
    ref = gy.float() @ w.float()
    err_b = float((dx.float() - ref).abs().max() / ref.abs().max())
    t_mine_b = timeit(lambda: K.gemm_bf16(gy, w, None, True, 0))
    t_lib_b = timeit(lambda: gy @ w)
    wt = w.t().contiguous()  # the engine's dX path: NT against W^T (ops/linear.py _w_t)
    t_mine_bt = timeit(lambda: K.gemm_bf16(gy, wt, None, False, 0))
    print(json.dumps({"gemm": name, "M": T, "N": N, "K": Kd,
                      "fwd_us": round(t_mine, 1), "fwd_TFs": round(flops / t_mine / 1e6, 1),
                      "fwd_lib_us": round(t_lib, 1), "fwd_lib_TFs": round(flops / t_lib / 1e6, 1), "fwd_relerr": err_f,
                      "dx_us": round(t_mine_b, 1), "dx_TFs": round(flops / t_mine_b / 1e6, 1),
                      "dx_nt_us": round(t_mine_bt, 1), "dx_nt_TFs": round(flops / t_mine_bt / 1e6, 1),
                      "dx_lib_us": round(t_lib_b, 1), "dx_lib_TFs": round(flops / t_lib_b / 1e6, 1),
                      "dx_relerr": err_b}), flush=True)
