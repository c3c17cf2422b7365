"""rocprofv3 probe: bf16 weight gradient with / without the fused bias at the GPT-2 shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from simple_distributed_machine_learning_amd import _native  # noqa: E402

K = _native.kernels()
dev = torch.device("cuda", 0)
T = 16384
for (inf, outf) in ((768, 2304), (3072, 768), (768, 3072)):
    x = torch.randn(T, inf, device=dev, dtype=torch.bfloat16)
    gy = torch.randn(T, outf, device=dev, dtype=torch.bfloat16)
    gw = torch.zeros(outf, inf, device=dev, dtype=torch.bfloat16)
    gb = torch.zeros(outf, device=dev, dtype=torch.bfloat16)
    order = os.environ.get("PROBE_ORDER", "ab")
    for mode in order:
        for _ in range(10):
            if mode == "a":
                K.wgrad_bf16_(gy, x, gw)
            else:
                K.wgrad_bf16_(gy, x, gw, gb)
        torch.cuda.synchronize()
print("done")
