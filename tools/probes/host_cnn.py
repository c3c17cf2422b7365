"""Host cost of one reference-CNN step at B = 60 (bench_configs ref_cnn): enqueue time with the device idle, and a
cProfile of the step's Python."""
import cProfile
import pstats
import time

import torch

from simple_distributed_machine_learning_amd.data import SyntheticMNIST
from simple_distributed_machine_learning_amd.models import get_model_spec
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

mesh = init_mesh(pp=2, schedule_kind="1f1b", rank=0, world_size=1)
dev = mesh.device
eng = PipelineEngine(get_model_spec("ref_cnn", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.01,
                     momentum=0.5, seed=1)
eng.train()
B = 60
ds = SyntheticMNIST(B * 2, seed=5, device=dev)


def step(i):
    return eng.run(ds, (i % 2) * B, B, train=True, global_batch=B)


for i in range(20):
    step(i)
torch.cuda.synchronize()
host = []
for i in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(i)
    host.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("host us per step (device idle at entry):", sorted(round(x, 1) for x in host))
pr = cProfile.Profile()
for i in range(200):
    pr.enable()
    step(i)
    pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
