"""Phase timing of the fused reference-CNN sample kernel (ref_cnn.hip cnn_step_sample_kernel) from its
s_memtime stamps: median over the 60 workgroups of the cycles between consecutive barriers."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from simple_distributed_machine_learning_amd import ops  # noqa: E402
from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402
from simple_distributed_machine_learning_amd._native import kernels  # noqa: E402

dev = torch.device("cuda", 0)
mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=dev)
e = PipelineEngine(get_model_spec("ref_cnn", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.1,
                   momentum=0.5, seed=3)
ds = SyntheticMNIST(600, seed=9, device=dev)
for i in range(20):
    e.run(ds, 0, 60, train=True)
torch.cuda.synchronize()
s0, s1 = e.stages[0], e.stages[1]
params = [s0.conv1.weight, s0.conv1.bias, s0.conv2.weight, s0.conv2.bias, s1.fc1.weight, s1.fc1.bias,
          s1.fc2.weight, s1.fc2.bias]
bufs = [e.optimizer.buffer_view(p) for p in params]
x = ds.inputs(0, 60).contiguous().float()
t = ds.targets(0, 60).contiguous()
stats = torch.empty(2, device=dev)
stamps = torch.zeros(60 * 16, dtype=torch.int64, device=dev)
res = []
for it in range(10):
    kernels().ref_cnn_step(x, t, [p.data for p in params], bufs, 1, 2, e.step_ctr, 0.5, True, 0.5, True, 1 / 60,
                           0.0, 0.5, 0.0, 0.0, False, False, stats, stamps)
    torch.cuda.synchronize()
    st = stamps.view(60, 16).cpu()
    res.append(st)
st = torch.stack(res[2:])  # [iters, 60, 16]
idx = [k for k in range(16) if int(st[0, 0, k]) != 0]
for a, b in zip(idx, idx[1:]):
    d = (st[:, :, b] - st[:, :, a]).double()
    print(f"phase {a:2d}->{b:2d}: median {float(d.median()):8.0f} cycles, max {float(d.max()):8.0f}")
tot = (st[:, :, idx[-1]] - st[:, :, idx[0]]).double()
print("total median", float(tot.median()), "cycles")
