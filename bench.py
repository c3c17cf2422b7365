"""Headline benchmark: samples/s (whole node) of the 2-stage MNIST-shape MLP (784->128->10).

BASELINE.json metric: "samples/sec (whole node), 2-stage MLP on MNIST-shape synthetic at
1/2/4/8 GPUs". The model is always cut into its 2 pipeline stages (fc1+ReLU | fc2 +
log_softmax + NLL), trained with SGD(lr 0.1, momentum 0.5) in fp32 — the reference's
optimizer and precision (/root/reference/simple_distributed.py:18-21, :100-104).

Placement by GPU count (weak scaling: per-GPU work is fixed at --batch_per_gpu samples):
  N=1   both stages on the one GPU (local hand-off, no p2p)
  N>=2  Chimera bidirectional 2-stage pipeline on each GPU pair (activations/grads over RCCL
        p2p on the pair's xGMI link) x dp = N/2 replicas (gradient all-reduce over RCCL)

Timing contract: W untimed warm-up steps; barrier + device sync; K timed steps (each a full
forward + backward + gradient sync + optimizer step over fresh data); barrier + device sync;
the MAX elapsed over ranks; rank 0 prints one JSON line.

    python bench.py --gpus 1 --steps 50 --warmup 10
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 50 --warmup 10
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from simple_distributed_machine_learning_amd.data import SyntheticMNIST
from simple_distributed_machine_learning_amd.models import get_model_spec
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

# reference RPC mechanism with the same 2-stage MLP on 8 vCPUs; the best number
# it reports for this model is 413,862 samples/s (B=4096, TCP-only transport). The headline
# B=60 figure is 13,704 samples/s. We compare against the stronger of the two.
BASELINE_SAMPLES_PER_S = 413_862.0
BASELINE_NOTE = "BASELINE.md 2-stage MLP, B=4096 TCP-only: 413,862 samples/s (B=60: 13,704)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch_per_gpu", type=int, default=int(os.environ.get("SDML_BENCH_BATCH", 65536)))
    p.add_argument("--microbatches", type=int, default=None, help="per pipeline (default: 1 on N=1, 4 chimera)")
    p.add_argument("--schedule", default=None, help="default: none on N=1, chimera on N>=2")
    p.add_argument("--dataset_batches", type=int, default=8, help="distinct batches cycled through")
    p.add_argument("--model", default="mlp")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        if rank == 0:
            print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    n = world
    if n == 1:
        kind, pp = (a.schedule or "1f1b"), 1
        M = a.microbatches or 1
    else:
        kind = a.schedule or "chimera"
        pp = 2
        M = a.microbatches or 4
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mesh = init_mesh(pp=pp, schedule_kind=kind, timeout_s=900, rank=rank, world_size=world)
    dev = mesh.device
    spec = get_model_spec(a.model, 2)
    engine = PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.1, momentum=0.5, seed=1)
    engine.train()
    # weak scaling: each pipeline replica processes batch_per_gpu * pp samples per step
    B = a.batch_per_gpu * pp
    GB = B * mesh.dp
    ds = SyntheticMNIST(B * a.dataset_batches, seed=1234, device=dev, offset=mesh.dp_rank * B * a.dataset_batches)

    def step(i):
        start = (i % a.dataset_batches) * B
        return engine.run(ds, start, B, train=True, global_batch=GB)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if world > 1:
            if dev.type == "cuda":
                dist.barrier(device_ids=[dev.index])
            else:
                dist.barrier()

    for i in range(a.warmup):
        step(i)
    sync()
    t0 = time.perf_counter()
    res = None
    for i in range(a.steps):
        res = step(a.warmup + i)
    sync()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    loss = None
    if res is not None:
        l, c, cnt = engine.reduce_metrics(res)
        loss = l / max(1, cnt)
    sps = GB * a.steps / el
    if rank == 0:
        out = {
            "metric": "samples/sec (whole node), 2-stage MLP on MNIST-shape synthetic",
            "value": round(sps, 1),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(sps / BASELINE_SAMPLES_PER_S, 2),
            "dtype": "fp32",
            "data": "synthetic (on-device MNIST-shape, random-init weights)",
            "config": {
                "model": "mlp-784-128-10 (2 pipeline stages)",
                "global_batch": GB,
                "seq_len": None,
                "parallelism": (f"pp2-chimera x dp{mesh.dp}" if pp == 2 else "single-GPU, both stages local"),
                "microbatches_per_pipeline": M,
                "batch_per_gpu": a.batch_per_gpu,
                "optimizer": "SGD lr=0.1 momentum=0.5",
            },
            "baseline": BASELINE_NOTE,
            "final_loss": None if loss is None else round(loss, 5),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        sync()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
