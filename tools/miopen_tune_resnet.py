"""Populate a MIOpen find-db for the ResNet-18 stage convolutions (torch.backends.cudnn.benchmark
= exhaustive MIOpen search) under MIOPEN_USER_DB_PATH, printing progress per step.

    MIOPEN_USER_DB_PATH=<dir> python tools/miopen_tune_resnet.py [--dtype bf16] [--batch 512]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="fp32")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=6)
a = ap.parse_args()
torch.backends.cudnn.benchmark = True
dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1)
eng = PipelineEngine(get_model_spec("resnet18", 8, dtype=dt), mesh, schedule_kind="1f1b", num_microbatches=1,
                     lr=0.01, momentum=0.5)
ds = SyntheticMNIST(a.batch * 2, seed=5, device=mesh.device)
for i in range(a.steps):
    t0 = time.perf_counter()
    eng.run(ds, (i % 2) * a.batch, a.batch, train=True)
    torch.cuda.synchronize()
    print(f"step {i}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
