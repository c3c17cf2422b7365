"""Where the GPT-2 step's device-to-device copies come from (torch.profiler, aten::copy_ / aten::cat call stacks)."""
import sys
import os

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

with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    eng.run(ds, 0, B, train=True, global_batch=B)
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
rows = [e for e in ka if e.key in ("aten::copy_", "aten::cat", "aten::contiguous", "aten::clone", "aten::to",
                                   "aten::_to_copy", "aten::add", "aten::add_", "aten::zero_", "aten::fill_",
                                   "aten::reshape", "aten::empty_like")]
rows.sort(key=lambda e: -e.count)
for e in rows[:30]:
    print(e.key, e.count, e.input_shapes)
# who calls copy_: the parents in the event tree
import collections
par = collections.Counter()
for ev in prof.events():
    if ev.name == "aten::copy_":
        p = ev.cpu_parent
        chain = []
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        par[" <- ".join(chain)] += 1
for k, v in par.most_common(15):
    print(v, k)
