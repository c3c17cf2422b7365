"""Training driver: train/test loops with the reference's log lines.

Reference flow (/root/reference/simple_distributed.py:86-136): rank 0 ("master") owns the
data, the model's first half, the loss and the logs; rank 1 ("worker1") only serves RPCs.
Here every rank runs this same driver (SPMD); rank 0 prints the identical lines:

    Train Epoch: 1 [0/6000 (0%)]\tLoss: 2.302585
    ...
    \nTest set: Average loss: 2.3026, Accuracy: 98/1000 (10%)\n

``python -m simple_distributed_machine_learning_amd.train --rank 0 --world_size 2 \
  --interface lo --master_addr 127.0.0.1 --master_port 29500`` (and rank 1 alike), or
under ``torchrun``.
"""
from __future__ import annotations

import os
import sys
import time
from typing import List, Optional

import torch

from . import cli
from .data import IdxMNIST, SyntheticMNIST, SyntheticTokens, batch_ranges
from .models import DEFAULT_STAGES, get_model_spec
from .parallel import PipelineEngine, init_mesh, shutdown
from .utils.checkpoint import load_checkpoint, save_checkpoint
from .utils.failure import Heartbeat
from .utils.metrics import JsonlMetrics, test_line, train_line


def _device(args) -> torch.device:
    if args.device == "cpu" or (args.device == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    local = int(os.environ.get("LOCAL_RANK", args.rank))
    n = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(1, n))
    torch.cuda.set_device(dev)
    return dev


def make_datasets(args, spec, device):
    if spec.input_kind == "tokens":
        S = spec.seq_len or args.seq_len or 64
        vocab = spec.vocab_size or 50257
        tr = SyntheticTokens(args.train_size, S, vocab, seed=args.data_seed, device=device)
        te = SyntheticTokens(args.test_size, S, vocab, seed=args.data_seed + 1, device=device)
        return tr, te
    use_mnist = args.data == "mnist" or (args.data == "auto" and IdxMNIST.available(args.data_dir))
    if use_mnist:
        px = getattr(args, "pixels", "f32")
        return (IdxMNIST(args.data_dir, True, device, pixels=px), IdxMNIST(args.data_dir, False, device, pixels=px))
    mode = "random" if args.data == "random" else "learnable"
    px = getattr(args, "pixels", "f32")
    tr = SyntheticMNIST(args.train_size, seed=args.data_seed, device=device, mode=mode, offset=0, pixels=px)
    te = SyntheticMNIST(args.test_size, seed=args.data_seed, device=device, mode=mode, offset=10_000_000, pixels=px)
    return tr, te


def run(args) -> dict:
    cli.export_env(args)
    device = _device(args)
    stages = args.stages or DEFAULT_STAGES[args.model]
    tp = max(1, getattr(args, "tp", 1))
    pp = args.pp or (2 if args.schedule == "chimera" else min(stages, args.world_size // tp))
    pp = max(1, min(pp, args.world_size // tp))
    while stages % pp:
        pp -= 1
    backend = None if args.backend == "auto" else args.backend
    mesh = init_mesh(pp=pp, schedule_kind=args.schedule, backend=backend, timeout_s=args.timeout,
                     rank=args.rank, world_size=args.world_size, device=device, tp=tp)
    hb = None
    if args.heartbeat > 0 and mesh.world_size > 1:
        hb = Heartbeat(mesh.rank, range(mesh.world_size), timeout_s=args.heartbeat).start()
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}.get(getattr(args, "dtype", "auto"))
    if dt is None and args.model == "resnet18" and device.type == "cuda":
        dt = torch.bfloat16  # the ResNet's GPU kernels are bf16 channels-last (ops/conv.py); fp32 is the CPU path
    kw = {"dtype": dt} if dt is not None and args.model in ("resnet18", "gpt2_tiny") else {}
    spec = get_model_spec(args.model, stages, eval_dropout=bool(args.eval_dropout), seq_len=args.seq_len,
                          dropout=getattr(args, "dropout", 0.5), **kw)
    if dt is not None and spec.param_dtype != dt:
        raise SystemExit(f"--dtype {args.dtype} is not supported for --model {args.model}")
    engine = PipelineEngine(spec, mesh, schedule_kind=args.schedule, num_microbatches=args.microbatches,
                            lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay, seed=args.seed,
                            debug_sync=args.debug_sync, timing=getattr(args, "timing", False))
    torch.manual_seed(args.seed * 7 + mesh.rank)  # dropout streams (reference: unseeded)
    if spec.input_kind == "tokens" and device.type == "cuda" and os.environ.get("SDML_GPT2_GEMM") == "lib":
        from .utils.tuned_gemm import use_tuned_gemms

        use_tuned_gemms()  # A/B only: the library GEMMs with the committed hipBLASLt solution table (TunableOp replay)
    train_ds, test_ds = make_datasets(args, spec, device)
    metrics = JsonlMetrics(args.metrics if mesh.is_master() else None, mesh.rank)
    master = mesh.is_master()
    B = args.batch_size
    GB = B * engine.data_shards  # one optimizer step consumes this many samples
    TB = args.test_batch_size or B
    start_epoch, start_batch = 1, 0
    if args.resume and args.ckpt_dir and os.path.exists(os.path.join(args.ckpt_dir, "stage0.pt")):
        meta = load_checkpoint(engine, args.ckpt_dir)
        start_epoch = max(1, meta["epoch"])
        start_batch = meta["batch"] + 1
        nb = (len(train_ds) + GB - 1) // GB
        if start_batch >= nb:
            start_epoch, start_batch = start_epoch + 1, 0
        if master:
            print(f"[sdml] resumed from {args.ckpt_dir}: epoch {start_epoch} batch {start_batch}", flush=True)

    history = {"train": [], "test": []}
    graphed = None
    if getattr(args, "graph", False) and device.type == "cuda" and not args.debug_sync:
        from .parallel.graphs import GraphedStep

        try:
            graphed = GraphedStep(engine, allow_collectives=os.environ.get("SDML_GRAPH_COLLECTIVES") == "1")
        except ValueError as e:
            if master:
                print(f"[sdml] --graph ignored: {e}", flush=True)

    def train(epoch: int, first_batch: int):
        engine.train()
        nb = (len(train_ds) + GB - 1) // GB
        t_last, n_since = time.perf_counter(), 0
        last_idx = first_batch - 1
        for batch_idx, start, size in batch_ranges(len(train_ds), GB, first_batch):
            if args.max_steps and batch_idx - first_batch >= args.max_steps:
                break
            if engine.data_shards > 1 and size < GB:
                # ragged last batch: shrink the per-shard batch (rotate needs equal shards)
                local = size // engine.data_shards
                if local == 0:
                    break
                size = local * engine.data_shards
            else:
                local = B
            if graphed is not None:
                res = graphed(train_ds, engine.local_start(start, local), local, global_batch=size)
            else:
                res = engine.run(train_ds, engine.local_start(start, local), local, train=True, global_batch=size)
            n_since += size
            last_idx = batch_idx
            if batch_idx % args.log_interval == 0:
                loss_sum, correct, cnt = engine.reduce_metrics(res)
                loss = loss_sum / max(1, cnt)
                now = time.perf_counter()
                sps = n_since / max(now - t_last, 1e-9)
                t_last, n_since = now, 0
                if master:
                    print(train_line(epoch, batch_idx, size, len(train_ds), nb, loss),
                          flush=True)
                    extra = {"timing_ms": engine.last_timing} if engine.timing else {}
                    metrics.log(event="train", epoch=epoch, batch=batch_idx, loss=loss, samples_per_s=sps, **extra)
                history["train"].append((epoch, batch_idx, loss))
        return last_idx

    def test():
        engine.eval()
        tot_loss, tot_correct, tot = 0.0, 0, 0
        for _, start, size in batch_ranges(len(test_ds), TB * engine.data_shards):
            local = TB if size == TB * engine.data_shards else size // engine.data_shards
            if local == 0:
                continue
            res = engine.run(test_ds, engine.local_start(start, local), local, train=False)
            l, c, n = engine.reduce_metrics(res)
            tot_loss += l
            tot_correct += c
            tot += n
        # divide by what was evaluated: with several data shards a ragged last test batch can
        # leave up to shards-1 samples out (the reference divides by len(test_ds) = the count
        # it evaluated, /root/reference/simple_distributed.py:129-132)
        n_ds = tot
        avg = tot_loss / max(1, n_ds)
        if master:
            print(test_line(avg, tot_correct, n_ds), flush=True)
            metrics.log(event="test", loss=avg, correct=tot_correct, n=n_ds)
        history["test"].append((avg, tot_correct, n_ds))

    prof = None
    if args.profile:
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if device.type == "cuda" else [])
        prof = profile(activities=acts)
        prof.__enter__()
    finished = False
    try:
        for epoch in range(start_epoch, args.epochs + 1):
            last = train(epoch, start_batch if epoch == start_epoch else 0)
            if not args.no_test:
                test()
            if args.ckpt_dir and (args.save_every and epoch % args.save_every == 0 or epoch == args.epochs):
                save_checkpoint(engine, args.ckpt_dir, epoch, last)
        finished = True
    finally:
        if prof is not None:
            prof.__exit__(None, None, None)
            if master:
                prof.export_chrome_trace(args.profile)
        if hb is not None:
            hb.stop(clean=finished)  # a rank that raised stays silent, so its peers abort
    history["engine"] = engine
    history["mesh"] = mesh
    return history


def main(argv: Optional[List[str]] = None) -> int:
    args = cli.parse_args(argv)
    hist = run(args)
    shutdown(hist["mesh"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
