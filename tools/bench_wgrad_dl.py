"""Time the rotate placement's stage-0 backward from the factored boundary gradient: head_dx_from_dl
+ linear_wgrad_u8 (dz written and read back) vs linear_wgrad_u8_dl (dz expanded in the kernel), and
the weight-gradient kernels alone (each including the slab reduction): dz given with a bound,
dl given with a bound (what the fused head attaches), dl without (workgroup-local bound)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import ops  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    N, Kd, C = 128, 784, 10
    out = {}
    for M in (65536, 131072):
        x8 = torch.randint(0, 256, (M, Kd), dtype=torch.uint8, device=dev)
        h = torch.randn(M, N, device=dev).relu_()
        dl = torch.randn(M, C, device=dev) * 1e-3
        w2 = torch.randn(C, N, device=dev) * 0.1
        buf = torch.zeros(N * Kd + N, device=dev)
        gw, gb = buf[:N * Kd].view(N, Kd), buf[N * Kd:]
        out[f"M{M}_unfused_us"] = round(timed(lambda: ops.linear_wgrad_u8(
            x8, ops.head_dx_from_dlogits(dl, w2, h, mask=True), gw, gb)), 1)
        out[f"M{M}_fused_us"] = round(timed(lambda: ops.linear_wgrad_u8_dl(x8, dl, w2, h, gw, gb)), 1)
        dz = ops.head_dx_from_dlogits(dl, w2, h, mask=True)
        am = dz.abs().amax().reshape(1)
        out[f"M{M}_dz_bound_us"] = round(timed(lambda: ops.linear_wgrad_u8(x8, dz, gw, gb, amax=am)), 1)
        out[f"M{M}_dl_bound_us"] = round(timed(lambda: ops.linear_wgrad_u8_dl(x8, dl, w2, h, gw, gb, amax=am)), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
