"""Host + device cost of the one-launch reference-size MLP step (mlp_small.hip) versus the engine's
multi-kernel step at B = 60: times the bare op, the engine path, and prints per-step microseconds."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd import ops  # noqa: E402
from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 60))
mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=dev)
e = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.1, momentum=0.5)
ds = SyntheticMNIST(B * 100, seed=1, device=dev)


def bench(fn, n=300):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


x = ds.x[:B].reshape(B, -1).contiguous()
y = ds.y[:B].contiguous()
stats = torch.empty(2, device=dev)
fc1, fc2 = e.stages[0].layers()[0], e.stages[1].layers()[0]
bare = bench(lambda i: ops.mlp_small_step(x, y, fc1, fc2, e.optimizer, 1.0 / B, stats))
eng = bench(lambda i: e.run(ds, (i % 100) * B, B, train=True))
os.environ["SDML_SMALL_STEP"] = "0"
e2 = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.1, momentum=0.5)
multi = bench(lambda i: e2.run(ds, (i % 100) * B, B, train=True))
print(json.dumps({"B": B, "bare_op_us": round(bare, 1), "engine_small_step_us": round(eng, 1),
                  "engine_multi_kernel_us": round(multi, 1)}))
