"""The data-parallel step's gradient all-reduce, overlapped (SDML_DP_SPLIT=1, default) or not, on ONE GPU:
a one-rank RCCL process group with a mesh that keeps its collectives (init_mesh(force_collectives=True)),
the headline MLP at 131072 rows, the engine path the N > 1 benchmark runs with nothing crossing GPUs
(rotate all-to-all, fused forward+head, deferred head reduction, gradient all-reduce, SGD).

    python tools/bench_dp_split.py [--steps 50] [--warmup 10] [--modes 1,0] [--blocks 240]

One JSON line per mode. Under ``rocprofv3 --kernel-trace`` the trace shows the RCCL kernel of range 0's
all-reduce next to range 1's weight-gradient kernel (tools/overlap_report.py reads it)."""
import argparse
import datetime
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--modes", default="1,0")
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--graph", action="store_true", help="replay the step (collective included) from a HIP graph")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=120))
    mesh = init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1, device=dev, force_collectives=True)
    B = a.batch
    ds = SyntheticMNIST(B * 4, seed=1234, device=dev, pixels="u8")
    for mode in a.modes.split(","):
        eng = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=1, lr=0.1,
                             momentum=0.5, seed=1, cross_fraction=0.0)
        eng.dp_split = mode == "1"
        if a.blocks:
            eng.dp_split_blocks = a.blocks
        assert eng.grad_sync.enabled
        run = eng.run
        if a.graph:
            from simple_distributed_machine_learning_amd.parallel.graphs import GraphedStep

            g = GraphedStep(eng, allow_collectives=True, direct_data=True, max_direct=4)

            def run(ds_, st, b, train=True):
                return g(ds_, st, b)
        for i in range(a.warmup):
            run(ds, (i % 4) * B, B, train=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            res = run(ds, (i % 4) * B, B, train=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"graph": a.graph, "dp_split": eng.dp_split, "blocks": eng.dp_split_blocks, "split_steps": eng.dp_split_steps,
                          "ms_per_step": round(el / a.steps * 1e3, 4), "samples_per_s": round(B * a.steps / el, 1),
                          "loss": round(float(res.loss_sum) / res.count, 5), "collectives": eng.transport.ops}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
