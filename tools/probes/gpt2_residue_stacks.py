"""Where the GPT-2 step's remaining ATen kernels come from: one profiled step (CPU + device), ATen ops that launch
device work, grouped by their Python call stack (torch.profiler group_by_stack_n)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from simple_distributed_machine_learning_amd.data import SyntheticTokens  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

mesh = init_mesh(pp=2, schedule_kind="1f1b", rank=0, world_size=1)
spec = get_model_spec("gpt2", 2, seq_len=1024)
eng = PipelineEngine(spec, mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.01, momentum=0.5, seed=1)
B = 16
ds = SyntheticTokens(B * 2, 1024, 50257, seed=5, device=mesh.device)
for i in range(3):
    eng.run(ds, (i % 2) * B, B, train=True, global_batch=B)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    eng.run(ds, 0, B, train=True, global_batch=B)
    torch.cuda.synchronize()
names = ("aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::sum", "aten::sort", "aten::to",
         "aten::_to_copy", "aten::clone", "aten::cat", "aten::index", "aten::mul", "aten::div", "aten::ne", "aten::eq",
         "aten::argmax", "aten::masked_fill", "aten::zeros", "aten::ones", "aten::full", "aten::arange", "aten::item",
         "aten::_local_scalar_dense", "aten::unique", "aten::sub", "aten::max", "aten::stack", "aten::where")
ka = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ka if e.key in names]
rows.sort(key=lambda e: -e.count)
for e in rows:
    st = [s for s in e.stack if "simple_distributed" in s or "tools/" in s][:4]
    print(f"{e.key:28s} n={e.count:3d}  dev_us={e.device_time_total:8.1f}  " + " <- ".join(st))
print("--- device kernels / memcpy by name")
for e in sorted(prof.key_averages(), key=lambda e: -e.device_time_total)[:40]:
    if e.device_time_total > 0 and ("Memcpy" in e.key or "Memset" in e.key or "at::native" in e.key or "rocprim" in e.key):
        print(f"{e.key[:90]:90s} n={e.count:3d} dev_us={e.device_time_total:8.1f}")
