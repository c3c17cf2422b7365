"""Host cost of one headline step (bench.py's N = 1 engine): enqueue time with the device idle, and a cProfile
of the step's Python."""
import cProfile
import pstats
import time

import torch

from simple_distributed_machine_learning_amd.data import SyntheticMNIST
from simple_distributed_machine_learning_amd.models import get_model_spec
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

mesh = init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1)
dev = mesh.device
eng = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=1, lr=0.1,
                     momentum=0.5, seed=1)
eng.train()
B = 131072
ds = SyntheticMNIST(B * 4, seed=1234, device=dev, pixels="u8")


def step(i):
    return eng.run(ds, (i % 4) * B, B, train=True, global_batch=B)


for i in range(5):
    step(i)
torch.cuda.synchronize()
host = []
for i in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(i)
    host.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("host us per step (device idle at entry):", [round(x, 1) for x in host])
pr = cProfile.Profile()
for i in range(50):
    torch.cuda.synchronize()
    pr.enable()
    step(i)
    pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:30]  # (file, line, fn) -> (cc, nc, tt, ct, callers)
for (f, ln, fn), (cc, nc, tt, ct, _) in rows:
    print(f"{tt / 50 * 1e6:8.2f} us self {ct / 50 * 1e6:8.2f} us cum {nc / 50:6.1f} calls  {f.split('/')[-1]}:{ln} {fn}")
