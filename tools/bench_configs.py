"""Throughput of the BASELINE.json configs through the pipeline engine on the local GPU(s).

    python tools/bench_configs.py --config mlp4x1024|resnet18|gpt2|ref_cnn [--steps N]
    torchrun --nproc-per-node 4 tools/bench_configs.py --config mlp4x1024   # real pipeline

With one process all stages are local (same schedule, local hand-offs); under torchrun the
stages are placed on ranks (gpipe for mlp4x1024, 1f1b otherwise). Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_distributed_machine_learning_amd.data import SyntheticMNIST, SyntheticTokens  # noqa: E402
from simple_distributed_machine_learning_amd.models import DEFAULT_STAGES, get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

DEFAULTS = {  # model -> (schedule, micro-batches, batch, seq_len)
    "mlp4x1024": ("gpipe", 8, 65536, None),
    "resnet18": ("1f1b", 8, 512, None),
    "gpt2": ("1f1b", 4, 16, 1024),
    "ref_cnn": ("1f1b", 1, 60, None),
    "mlp": ("1f1b", 1, 60, None),  # the reference's own batch (13,704 samples/s at B=60)
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mlp4x1024", choices=sorted(DEFAULTS))
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 10; 200 for the batch-60 configs, whose ~0.06 ms steps need more)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3; 20 for the batch-60 configs)")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--seq_len", type=int, default=None)
    ap.add_argument("--graph", nargs="?", const="copy", default=None, choices=["copy", "direct"],
                    help="replay the step from a captured hipGraph (copy: static data buffers refilled per step; "
                         "direct: one graph per cycled batch reading the device-resident data in place)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel ranks per stage (gpt2)")
    ap.add_argument("--dtype", default=None, choices=[None, "fp32", "bf16"], help="resnet18: compute dtype")
    ap.add_argument("--pixels", default="auto", choices=["auto", "f32", "u8"],
                    help="image models: pixel storage (auto: uint8 for the MLPs at batches the uint8 kernels take)")
    a = ap.parse_args()
    kind, M, B, S = DEFAULTS[a.config]
    small = a.config in ("mlp", "ref_cnn") and (a.batch or B) <= 128
    if a.steps is None:
        a.steps = 200 if small else 10
    if a.warmup is None:
        a.warmup = 20 if small else 3
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    if world0 == 1 and a.config in ("gpt2", "resnet18", "mlp4x1024"):
        # all stages local: micro-batching only shrinks the GEMMs / convolutions (measured: GPT-2
        # 614K vs 438K tokens/s at M=4; ResNet-18 27.2K vs 15.6K samples/s at M=8; 4x1024 MLP
        # 6.27M vs 5.61M samples/s at M=8)
        M = 1
    M = a.microbatches or M
    B = a.batch or B
    if a.pixels == "auto":
        a.pixels = "u8" if a.config in ("mlp", "mlp4x1024") and B >= 4096 else "f32"
    S = a.seq_len or S
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    stages = DEFAULT_STAGES[a.config]
    pp = min(world // a.tp, stages)
    mesh = init_mesh(pp=pp, schedule_kind=kind, rank=rank, world_size=world, tp=a.tp)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}.get(a.dtype)
    if dt is None and a.config == "resnet18" and torch.cuda.is_available():
        # the hand-written conv / BatchNorm kernels are bf16 channels-last (fp32 runs on MIOpen):
        # 107K vs 27.2K samples/s on one MI355X
        dt = torch.bfloat16
    spec = get_model_spec(a.config, stages, seq_len=S, **({"dtype": dt} if dt is not None else {}))
    eng = PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.01, momentum=0.5, seed=1)
    tuned = False
    if spec.input_kind == "tokens" and mesh.device.type == "cuda" and os.environ.get("SDML_GPT2_GEMM") == "lib":
        from simple_distributed_machine_learning_amd.utils.tuned_gemm import use_tuned_gemms

        tuned = use_tuned_gemms()
    dev = mesh.device
    if dev.type == "cuda":
        from simple_distributed_machine_learning_amd import _native

        _native.apply_knobs_from_env()  # A/B runs only (SDML_KNOBS="NAME=V,..."); default: none
    nb = 2
    if spec.input_kind == "tokens":
        ds = SyntheticTokens(B * eng.data_shards * nb, S, 50257, seed=5, device=dev)
        unit = "tokens/s"
        per_sample = S
    else:
        ds = SyntheticMNIST(B * eng.data_shards * nb, seed=5, device=dev, pixels=a.pixels)
        unit = "samples/s"
        per_sample = 1
    GB = B * eng.data_shards

    graphed = None
    if a.graph:
        from simple_distributed_machine_learning_amd.parallel.graphs import GraphedStep

        graphed = GraphedStep(eng, direct_data=a.graph == "direct", max_direct=nb)

    def step(i):
        st = (i % nb) * GB
        if graphed is not None:
            return graphed(ds, eng.local_start(st, B), B, global_batch=GB)
        return eng.run(ds, eng.local_start(st, B), B, train=True, global_batch=GB)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for i in range(a.warmup):
        step(i)
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        res = step(i)
    sync()
    el = time.perf_counter() - t0
    l, c, n = eng.reduce_metrics(res)
    if rank == 0:
        print(json.dumps({"config": a.config, "schedule": kind, "stages": stages, "ranks": world, "tp": a.tp,
                          "microbatches": M, "batch": GB, "seq_len": S, "dtype": str(spec.param_dtype), "graph": a.graph or False, "tuned_gemms": tuned,
                          "pixels": a.pixels,
                          "value": round(GB * per_sample * a.steps / el, 1), "unit": unit,
                          "ms_per_step": round(el / a.steps * 1e3, 3), "loss": round(l / max(1, n), 4),
                          "bubble_model": round(eng.schedule(M, False).bubble_fraction(), 3)}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
