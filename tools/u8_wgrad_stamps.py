"""Phase timing of the uint8 weight gradient (mlp_u8.hip u8_wgrad_kernel<2>: ReLU bits + factored dl, the
headline step's second kernel, or u8_wgrad_ring_kernel when knob U8_WGRAD_RING is on - the default) at 131072 x 784
-> 128 from its s_memtime stamps (experiments build only). Ring kernel: "stage+gload+barrier" is the DMA wait + barrier
at the top of the next K-step, and the compute intervals include the next K-step's dz build and DMA issue.

Per (block, wave): 1 start, 2 after the dz-bound reduction, 3 after the prologue (first K-step staged), 4 / 5 after
K-step 0's compute / barrier, 6 / 7 the same for K-step 8, 8 / 9 for K-step 16, 10 after the last compute,
11 after the partial-tile stores, 12 end; 0 / 15 s_memrealtime at start / end."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import ops  # noqa: E402
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402

K = kernels()
M, N, KD, C = 131072, 128, 784, 10
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
x8 = torch.randint(0, 256, (M, KD), dtype=torch.uint8, device=dev, generator=g)
h = torch.rand(M, N, device=dev, generator=g) - 0.3
bits = ops.relu_bits(h)
dl = (torch.rand(M, C, device=dev, generator=g) - 0.5) * 1e-3
w2 = (torch.rand(C, N, device=dev, generator=g) - 0.5) * 0.2
gbuf = torch.zeros(N * KD + N, device=dev)


# the dz bound as the fused head hands it over in the headline step (one value per forward block)
amax = ((dl.abs().sum(1) * w2.abs().max() * 2).view(-1, 256).amax(1)).contiguous()


def run():
    ops.linear_wgrad_u8_dl(x8, dl, w2, bits, gbuf[:N * KD].view(N, KD), gbuf[N * KD:], amax=amax)


def timed(n=30):
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


if len(sys.argv) > 1:  # e.g. U8_WGRAD_RING=0
    name, v = sys.argv[1].split("=")
    K.set_knob(name, int(v))
plain = timed()
NB = 4096
stamps = torch.zeros(NB * 8 * 16, dtype=torch.int64, device=dev)
if not K.u8_set_wgrad_stamps(stamps):
    print(json.dumps({"error": "production build: no stamps", "plain_us_incl_reduction": round(plain, 1)}))
    sys.exit(0)
stamped = timed(10)
res = []
for _ in range(6):
    stamps.zero_()
    run()
    torch.cuda.synchronize()
    res.append(stamps.view(NB, 8, 16).cpu().clone())
K.u8_set_wgrad_stamps(None)
st = torch.stack(res[1:]).double()
used = st[0, :, 0, 1] != 0
st = st[:, used]
out = {"plain_us_incl_reduction": round(plain, 1), "stamped_us": round(stamped, 1), "blocks": int(used.sum())}
names = {(1, 2): "dz bound", (2, 3): "prologue (gload+stage 0, barrier)", (3, 4): "k0 compute",
         (4, 5): "k0 stage+gload+barrier", (5, 6): "k1..k8 compute (8 steps incl 7 syncs)", (6, 7): "k8 stage+barrier",
         (7, 8): "k9..k16 compute", (8, 9): "k16 stage+barrier", (9, 10): "k17..last", (10, 11): "tile stores",
         (11, 12): "bias partial + exit"}
for wv in (0, 1, 4):
    row = {}
    for (a, b), nm in names.items():
        row[nm] = round(float((st[:, :, wv, b] - st[:, :, wv, a]).median()), 0)
    row["total cycles"] = round(float((st[:, :, wv, 12] - st[:, :, wv, 1]).median()), 0)
    row["wall ns"] = round(float(((st[:, :, wv, 15] - st[:, :, wv, 0]) * 10).median()), 0)
    out[f"wave{wv}"] = row
t0 = st[:, :, :, 0].flatten(1).amin(1)
out["kernel span us"] = round(float(((st[:, :, :, 15].flatten(1).amax(1) - t0) * 0.01).median()), 2)
out["block start spread us"] = round(float(((st[:, :, 0, 0].amax(1) - t0) * 0.01).median()), 2)
print(json.dumps(out, indent=1))
