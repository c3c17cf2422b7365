"""Micro-benchmark of the uint8-pixel first-layer GEMMs at the headline shape (131072 x 784 -> 128).
Env knobs (read once per process): SDML_X3_DEEP, SDML_U8_WGRAD_WG_PER_CU, SDML_U8_FWD=x3, SDML_U8_WGRAD=x3."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
M, N, Kd = 131072, 128, 784
dev = torch.device("cuda", 0)
x8 = torch.randint(0, 256, (M, Kd), dtype=torch.uint8, device=dev)
w = torch.randn(N, Kd, device=dev) * 0.05
b = torch.randn(N, device=dev)
gz = torch.randn(M, N, device=dev)
_g = torch.zeros(N * Kd + N, device=dev)  # flat layout: gb right after gw (as in the engine's grad buffer)
gw, gb = _g[:N * Kd].view(N, Kd), _g[N * Kd:]


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


fwd = timeit(lambda: K.linear_fwd_u8(x8, w, b, True, 1.0 / 255.0))
wg = timeit(lambda: K.linear_wgrad_u8(x8, gz, gw, gb, 1.0 / 255.0))
print(json.dumps({"deep": os.environ.get("SDML_X3_DEEP", "1"), "wg_per_cu": os.environ.get("SDML_U8_WGRAD_WG_PER_CU", "1"),
                  "fwd_us": round(fwd, 1), "wgrad_us": round(wg, 1)}))
