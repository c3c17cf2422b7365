"""Phase timing of the reference CNN step's split backward kernel (ref_cnn.hip cnn_step_bwd_kernel, knob
CNN_SPLIT_BWD = 2 turns its s_memtime stamps on): medians over the B x 10 workgroups of the cycles between
its barriers, plus the spread of workgroup start / end times (s_memrealtime, 100 MHz) over the launch.
Phases: 0->1 global loads into LDS, 1->2 pool argmaxes, 2->3 dW2 / db2 + dZ1 quarters, 3->4 ReLU mask,
4->5 dW1 / db1."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402

B = 60
dev = torch.device("cuda", 0)
mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=dev)
e = PipelineEngine(get_model_spec("ref_cnn", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.1,
                   momentum=0.5, seed=3)
ds = SyntheticMNIST(600, seed=9, device=dev)
for i in range(20):
    e.run(ds, 0, B, train=True)
torch.cuda.synchronize()
s0, s1 = e.stages[0], e.stages[1]
params = [s0.conv1.weight, s0.conv1.bias, s0.conv2.weight, s0.conv2.bias, s1.fc1.weight, s1.fc1.bias,
          s1.fc2.weight, s1.fc2.bias]
bufs = [e.optimizer.buffer_view(p) for p in params]
x = ds.inputs(0, B).contiguous().float()
t = ds.targets(0, B).contiguous()
stats = torch.empty(2, device=dev)
K = kernels()
K.set_knob("CNN_SPLIT_BWD", 2)
stamps = torch.zeros(B * 10 * 16, dtype=torch.int64, device=dev)
res = []
for it in range(12):
    K.ref_cnn_step(x, t, [p.data for p in params], bufs, 1, 2, e.step_ctr, 0.5, True, 0.5, True, 1 / B,
                   0.0, 0.5, 0.0, 0.0, False, False, stats, stamps)
    torch.cuda.synchronize()
    res.append(stamps.view(B * 10, 16).cpu().clone())
K.reset_knobs()
st = torch.stack(res[2:]).double()  # [iters, blocks, 16]
out = {}
for a, b in zip(range(5), range(1, 6)):
    d = st[:, :, b] - st[:, :, a]
    out[f"phase {a}->{b} cycles"] = {"median": float(d.median()), "max": float(d.amax(1).median())}
tot = st[:, :, 5] - st[:, :, 0]
out["block total cycles"] = {"median": float(tot.median()), "max": float(tot.amax(1).median())}
t0 = st[:, :, 14].amin(1, keepdim=True)
out["block start spread us (median over iters of max-min)"] = float(((st[:, :, 14] - t0).amax(1) * 0.01).median())
out["block end us after first start"] = float(((st[:, :, 15] - t0).amax(1) * 0.01).median())
out["median block life us"] = float(((st[:, :, 15] - st[:, :, 14]) * 0.01).median())
print(json.dumps(out, indent=1))
