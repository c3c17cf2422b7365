"""Headline benchmark: samples/s (whole node) of the 2-stage MNIST-shape MLP (784->128->10).

BASELINE.json metric: "samples/sec (whole node), 2-stage MLP on MNIST-shape synthetic at
1/2/4/8 GPUs". The model is always cut into its 2 pipeline stages (fc1+ReLU | fc2 +
log_softmax + NLL), trained with SGD(lr 0.1, momentum 0.5) in fp32 — the reference's
optimizer and precision (/root/reference/simple_distributed.py:18-21, :100-104).

Placement ("rotate" pipeline; weak scaling: per-GPU work fixed at --batch_per_gpu samples):
  every GPU owns a data shard and hosts both stages; each step is cut into W waves and in
  every wave stage 0's output is split R ways and exchanged with ONE RCCL all-to-all (part k
  -> GPU k), stage 1 (+ loss + its backward) runs on what arrived, the input-gradients go
  back by the inverse all-to-all, stage 0 runs its backward; stage weights are replicated and
  their gradients all-reduced over RCCL. On an 8-GPU node every stage boundary therefore
  fans out over all 7 xGMI links of each GPU instead of one neighbour link. N=1 is the same
  code with the exchange elided (both stages local).
  (--schedule chimera / 1f1b select the classic neighbour pipelines instead.)

Data: synthetic MNIST-shape images stored as uint8 bytes, the way MNIST ships them (``--pixels u8``,
default). ToTensor's /255, which the reference runs on the host per batch
(/root/reference/simple_distributed.py:87-88), is folded into fc1's fp32-accurate GEMM (the bytes
are exact in fp16, the weights two fp16 planes within one fp32 ulp; README "uint8 pixels").
``--pixels f32`` stores float32 images instead.

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


class _ShardedSynth:
    """Per-rank view of the global synthetic dataset: labels for every sample, images only for
    the samples this rank's stage 0 consumes (``own_len`` samples at ``own_lo`` of each of the
    ``nbatches`` global batches of ``GB`` samples)."""

    def __init__(self, GB, own_lo, own_len, nbatches, dev, pixels="u8"):
        self.n = GB * nbatches
        self.GB, self.own_lo, self.own_len = GB, own_lo, own_len
        self.labels = SyntheticMNIST(self.n, seed=1234, device=dev, image_range=(0, 0))
        self.imgs = [SyntheticMNIST(own_len, seed=1234, device=dev, offset=k * GB + own_lo, pixels=pixels)
                     for k in range(nbatches)]

    def inputs(self, start, n):
        k, r = divmod(start, self.GB)
        r -= self.own_lo
        assert 0 <= r and r + n <= self.own_len, (start, n)
        return self.imgs[k].x[r:r + n]

    def targets(self, start, n):
        return self.labels.y[start:start + n]

    def __len__(self):
        return self.n


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch_per_gpu", type=int, default=int(os.environ.get("SDML_BENCH_BATCH", 131072)))
    p.add_argument("--waves", type=int, default=None, help="rotate: waves per step (default 1 on N=1, else 2)")
    p.add_argument("--microbatches", type=int, default=None, help="chimera/1f1b: micro-batches per pipeline")
    p.add_argument("--schedule", default="rotate", choices=["rotate", "chimera", "1f1b", "gpipe"])
    p.add_argument("--dataset_batches", type=int, default=4, help="distinct batches cycled through")
    p.add_argument("--model", default="mlp")
    p.add_argument("--pixels", default="u8", choices=["u8", "f32"],
                   help="image storage: MNIST's uint8 bytes (ToTensor's /255 fused into fc1) or float32")
    return p.parse_args()


def _parallelism(kind, n, mesh):
    if n == 1:
        return "single GPU, both pipeline stages local"
    if kind == "rotate":
        return f"pp2 rotate: {n} GPUs x (stage0+stage1), all-to-all stage boundary over RCCL/xGMI, grad all-reduce"
    return f"pp{mesh.pp}-{kind} x dp{mesh.dp}"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        if rank == 0:
            print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    n = world
    kind = a.schedule
    if kind == "rotate":
        pp = world
        W = a.waves or (1 if n == 1 else 2)
        M = W * pp
        B = a.batch_per_gpu  # per owner shard
    else:
        pp = 1 if n == 1 else 2
        M = a.microbatches or (1 if n == 1 else 4)
        B = a.batch_per_gpu * pp  # per pipeline replica
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # rotate on a 2-stage model runs its boundary as all-to-all collectives: no p2p channels
    mesh = init_mesh(pp=pp, schedule_kind=kind, timeout_s=900, rank=rank, world_size=world,
                     p2p_channels=(kind != "rotate"))
    dev = mesh.device
    spec = get_model_spec(a.model, 2)
    engine = PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.1, momentum=0.5, seed=1)
    engine.train()
    GB = B * engine.data_shards  # samples per optimizer step, whole node
    # fresh data every step, cycling over `dataset_batches` global batches; a rank
    # materialises images only for the shards it feeds into stage 0 (labels for all)
    if world == 1:
        ds = SyntheticMNIST(GB * a.dataset_batches, seed=1234, device=dev, pixels=a.pixels)
    else:  # rotate: own shard of the group block; chimera/1f1b: the replica's whole batch
        own_lo = engine.local_start(0, B) + (mesh.pp_rank * B if kind == "rotate" else 0)
        ds = _ShardedSynth(GB, own_lo, B, a.dataset_batches, dev, pixels=a.pixels)

    def step(i):
        start = (i % a.dataset_batches) * GB
        return engine.run(ds, engine.local_start(start, B), B, train=True, global_batch=GB)

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
            "data": ("synthetic (on-device MNIST-shape, random-init weights; "
                     + ("uint8 pixels as MNIST ships them, ToTensor /255 fused into fc1's fp32-accurate GEMM)"
                        if a.pixels == "u8" else "float32 pixels)")),
            "config": {
                "model": "mlp-784-128-10 (2 pipeline stages)",
                "global_batch": GB,
                "seq_len": None,
                "parallelism": _parallelism(kind, n, mesh),
                "microbatches": M,
                "batch_per_gpu": a.batch_per_gpu,
                "optimizer": "SGD lr=0.1 momentum=0.5",
                "pixels": a.pixels,
                "gemm_numerics": ("fp32-accurate: fp32 operands as exact hi+lo fp16 planes (within one fp32 ulp) "
                                  "or 3 bf16 planes, fp32 accumulation (README 'Two fp16 planes')"),
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
