"""Phase timing of the fused uint8 forward + classifier head (mlp_u8.hip u8_fwd_kernel<7, ...>) at the headline
shape from its s_memtime stamps. Needs the experiments build of _kernels (SDML_KERNEL_EXPERIMENTS=1); the
production build has no MODE 7 variant and this script exits.

Per (block, wave) the kernel stamps: 1 start, 2..13 after the barriers of K-steps 0..11, 15 after the K loop, 16 at
the head epilogue's entry, 17 after its first barrier (block max |h| exchanged: h, the ReLU bits and W2 in
registers), 18 after the second (the fp16 h image written), 19 logits / softmax / dl done, 20 after the third barrier
(dl^T image), 21 dW2 and the slab row written, 22 end; slots 0 / 23 hold s_memrealtime (100 MHz) at start / end
(head_block.h).
Prints medians over workgroups of each phase, split into the first and second round of workgroups (by start time).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import ops  # noqa: E402
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402

K = kernels()
from simple_distributed_machine_learning_amd import _native  # noqa: E402

_native.apply_knobs_from_env()  # SDML_KNOBS="U8_FH_STAGES=3,..." (A/B)
M, N, Kd, C = 131072, 128, 784, 10
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
x8 = torch.randint(0, 256, (M, Kd), dtype=torch.uint8, device=dev, generator=g)
w1 = torch.randn(N, Kd, device=dev, generator=g) * 0.05
b1 = torch.randn(N, device=dev, generator=g) * 0.1
w2 = torch.randn(C, N, device=dev, generator=g) * 0.1
b2 = torch.randn(C, device=dev, generator=g) * 0.1
tgt = torch.randint(0, C, (M,), device=dev, generator=g)
gw2, gb2 = torch.zeros(C, N, device=dev), torch.zeros(C, device=dev)
stats = torch.zeros(2, device=dev)
dl = torch.empty(M, C, device=dev)
mask = torch.empty(M, N // 32, dtype=torch.int32, device=dev)
cache = ops.PlaneCache(w1)
blocks = K.u8_fwd_head_blocks(M) if hasattr(K, 'u8_fwd_head_blocks') else (M + 255) // 256
S = K.u8_stamp_slots()
stamps = torch.zeros(blocks * 8 * S, dtype=torch.int64, device=dev)


def run():
    ops.linear_relu_head_u8(x8, w1, b1, cache, 0, w2, b2, tgt, gw2, gb2, 1.0 / M, stats, True, dl, mask)


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


plain_us = timed()
if os.environ.get("SDML_U8_FWD_MODE"):  # a timing variant (experiments build): its time only
    print(json.dumps({"mode": os.environ["SDML_U8_FWD_MODE"], "us": round(plain_us, 1)}))
    sys.exit(0)
if not K.u8_set_stamps(stamps):
    print(json.dumps({"error": "production build: no stamp variant", "plain_us": round(plain_us, 1)}))
    sys.exit(0)
stamped_us = timed(10)
res = []
for it in range(6):
    run()
    torch.cuda.synchronize()
    res.append(stamps.view(blocks, 8, S).cpu().clone())
K.u8_set_stamps(None)
st = torch.stack(res[1:]).double()  # [iters, blocks, waves, S]
start_rt = st[:, :, 0, 0]  # wave 0 realtime start per block
out = {"plain_us": round(plain_us, 1), "stamped_us": round(stamped_us, 1)}
# rounds: blocks ranked by start time within each iteration; first 256 = round 0
order = start_rt.argsort(dim=1)
rank = torch.empty_like(order)
rank.scatter_(1, order, torch.arange(blocks).expand_as(order))
rnd = (rank >= 256).double()
names = {(1, 2): "prologue", (2, 13): "k-steps 0..11 (11 intervals)", (13, 15): "k-steps 11, 12 + tail",
         (15, 16): "to epilogue", (16, 17): "h, mask, W2, max + barrier", (17, 18): "h image + barrier",
         (18, 19): "logits/softmax/dl", (19, 20): "barrier", (20, 21): "dW2 + slab", (21, 22): "exit"}
for wv in (0, 4, 7):
    for r in (0, 1):
        sel = rnd == r
        row = {}
        for (a, b), nm in names.items():
            d = (st[:, :, wv, b] - st[:, :, wv, a])[sel]
            row[nm] = round(float(d.median()), 0)
        tot = (st[:, :, wv, 22] - st[:, :, wv, 1])[sel]
        row["total cycles"] = round(float(tot.median()), 0)
        wall = (st[:, :, wv, 23] - st[:, :, wv, 0])[sel] * 10.0  # ns
        row["wall ns"] = round(float(wall.median()), 0)
        out[f"wave{wv}_round{r}"] = row
# per-K-step intervals of wave 0, round 0 (cycles)
ks = [round(float((st[:, :, 0, k + 1] - st[:, :, 0, k])[rnd == 0].median()), 0) for k in range(2, 13)]
out["wave0_round0_kstep_cycles"] = ks
# kernel span and round boundaries (realtime, ns)
t0 = st[:, :, :, 0].amin(dim=(1, 2), keepdim=False)
t1 = st[:, :, :, 23].amax(dim=(1, 2))
out["kernel_span_us"] = round(float(((t1 - t0) * 10.0 / 1e3).median()), 2)
r0_end = torch.stack([st[i, :, :, 23][rnd[i] == 0].amax() for i in range(st.shape[0])])
r1_start = torch.stack([st[i, :, :, 0][rnd[i] == 1].amin() for i in range(st.shape[0])])
out["round0_end_us"] = round(float(((r0_end - t0) * 10.0 / 1e3).median()), 2)
out["round1_first_start_us"] = round(float(((r1_start - t0) * 10.0 / 1e3).median()), 2)
print(json.dumps(out, indent=1))
