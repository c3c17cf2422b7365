"""Headline benchmark: samples/s (whole node) of the 2-stage MNIST-shape MLP (784->128->10).

BASELINE.json metric: "samples/sec (whole node), 2-stage MLP on MNIST-shape synthetic at
1/2/4/8 GPUs". The model is always cut into its 2 pipeline stages (fc1+ReLU | fc2 +
log_softmax + NLL), trained with SGD(lr 0.1, momentum 0.5) in fp32 — the reference's
optimizer and precision (/root/reference/simple_distributed.py:18-21, :100-104).

Placement (``--placement``, parallel/placement.py; weak scaling: per-GPU work fixed at
--batch_per_gpu samples): N = 1 runs both stages on the one GPU. For N > 1 the placement is a
decision of the link/compute cost model, not a default:
  pp2dp     the reference's cut replicated: GPU pairs (stage 0 | stage 1), Chimera schedule,
            boundary tensors by RCCL isend/irecv over the pair's xGMI link, dp over the pairs
  rotate    every GPU owns a shard and hosts both stages; an equal share of each wave's boundary
            goes to every peer with ONE RCCL all-to-all per wave and direction (all 7 links)
  balanced  rotate with the cross-GPU fraction sized so the links stay under the compute
  dp        rows stay on their owner (nothing crosses); gradients all-reduced
  auto      (default) the fastest predicted placement; within 2 %, the one moving the most
            boundary bytes across GPUs
The JSON ``config`` carries the placement, the boundary bytes that crossed GPUs per step
(measured by the transport), the link model and every placement's prediction.

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
import subprocess
import sys
import time

import torch
import torch.distributed as dist

from simple_distributed_machine_learning_amd.data import SyntheticMNIST
from simple_distributed_machine_learning_amd.models import get_model_spec
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh
from simple_distributed_machine_learning_amd.parallel import placement as plc

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
    p.add_argument("--placement", default="auto", choices=plc.PLACEMENTS,
                   help="where the two stages run on N GPUs (parallel/placement.py)")
    p.add_argument("--cross_fraction", type=float, default=None,
                   help="rotate family: fraction of each wave whose stage 1 runs on a peer (overrides the model)")
    p.add_argument("--waves", type=int, default=None,
                   help="rotate family: waves per step (default 1 when nothing crosses GPUs, else 2)")
    p.add_argument("--microbatches", type=int, default=None, help="pp2dp: micro-batches per pipeline")
    p.add_argument("--schedule", default=None, choices=["chimera", "1f1b", "gpipe"],
                   help="pp2dp: pipeline schedule (default chimera)")
    p.add_argument("--dataset_batches", type=int, default=4, help="distinct batches cycled through")
    p.add_argument("--model", default="mlp")
    p.add_argument("--alternatives", default="auto", choices=["auto", "on", "off"],
                   help="after the timed steps, also time the reference's placement (pp2dp) for the JSON; "
                        "auto: at every even N (the reference's cut at 2, 4, 8 GPUs)")
    p.add_argument("--link_probe", default="auto", choices=["auto", "on", "off"],
                   help="N > 1: measure the all-reduce / all-to-all / pair exchange on the job's process group before "
                        "choosing the placement, and feed the measured link model to it (parallel/linkprobe.py)")
    p.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                   help="replay each step from a HIP graph (parallel/graphs.py, one graph per cycled batch reading "
                        "the device-resident data in place, the gradient all-reduce inside); auto: on for the dp "
                        "placement over RCCL at N > 1, off at N = 1 (measured, README 'HIP graphs')")
    p.add_argument("--pixels", default="u8", choices=["u8", "f32"],
                   help="image storage: MNIST's uint8 bytes (ToTensor's /255 fused into fc1) or float32")
    return p.parse_args()


def _parallelism(placement, n, mesh, phi, kind):
    if n == 1:
        return "single GPU, both pipeline stages local"
    if placement == "pp2dp":
        return f"pp2 x dp{mesh.dp}: GPU pairs (stage0 | stage1), {kind} schedule, RCCL isend/irecv over xGMI"
    if phi == 0:
        return f"dp{n}: both stages on every GPU, no boundary crosses GPUs, RCCL gradient all-reduce"
    share = "equal shares" if phi is None else f"{phi:.4g} of each wave"
    return (f"pp2 {placement}: {n} GPUs x (stage0+stage1), stage-1 rows on peers ({share}) by RCCL all-to-all "
            f"over xGMI, gradient all-reduce")


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(n: int) -> int:
    """``--gpus N > 1`` without a launcher: start the N ranks as child processes (one per GPU,
    torch.distributed.run on 127.0.0.1) BEFORE anything in this process touches the GPU, relay their
    output and return rank 0's exit status. ``torch.cuda.device_count()`` does not initialise the
    GPU on this image, so it is safe to check here; the host-staged transport (SDML_TRANSPORT=host)
    lets N ranks share fewer GPUs."""
    host_staged = os.environ.get("SDML_TRANSPORT") == "host"
    have = torch.cuda.device_count()
    if not host_staged and 0 < have < n:  # (no GPU at all: the CPU/Gloo rehearsal)
        print(f"[bench] --gpus {n} but only {have} GPU(s) visible (SDML_TRANSPORT=host shares one GPU)",
              file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ, SDML_BENCH_LAUNCHED="1")
    return subprocess.run(cmd, env=env).returncode


def _measure_pp2dp(a, n, rank, world, dev, steps=10, warmup=3):
    """The reference's own placement (stage 0 | stage 1 on different GPUs of a pair, Chimera, dp over the
    pairs), timed for a few steps AFTER the headline measurement so the JSON carries a measured number
    for it next to the placement the model chose (same per-GPU batch, weak scaling)."""
    mesh = init_mesh(pp=2, schedule_kind="chimera", timeout_s=900, rank=rank, world_size=world, p2p_channels=True)
    spec = get_model_spec(a.model, 2)
    eng = PipelineEngine(spec, mesh, schedule_kind="chimera", num_microbatches=4, lr=0.1, momentum=0.5, seed=1)
    eng.train()
    B = a.batch_per_gpu * 2
    GB = B * eng.data_shards
    own_lo = eng.local_start(0, B)
    ds = _ShardedSynth(GB, own_lo, B, 2, dev, pixels=a.pixels)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        mesh.barrier()

    for i in range(warmup):
        eng.run(ds, eng.local_start((i % 2) * GB, B), B, train=True, global_batch=GB)
    sync()
    eng.transport.reset_counters()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.run(ds, eng.local_start((i % 2) * GB, B), B, train=True, global_batch=GB)
    sync()
    t = torch.tensor([time.perf_counter() - t0, float(eng.transport.bytes_sent)], dtype=torch.float64, device=dev)
    tmax = t[:1].clone()
    eng.transport.all_reduce(tmax, channel="world", op=dist.ReduceOp.MAX, async_op=False)
    eng.transport.all_reduce(t, channel="world", async_op=False)
    el = float(tmax.item())
    return {"placement": "pp2dp", "schedule": "chimera", "microbatches": 4, "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 4), "samples_per_s": round(GB * steps / el, 1),
            "boundary_bytes_across_gpus_per_step": int(float(t[1].item()) / steps),
            "predicted": plc.predict("pp2dp", n, a.batch_per_gpu)}


def _replica_check(engine, mesh, dev, rank):
    """After the timed steps: every replica of a stage must hold bit-identical parameters (the gradient all-reduce
    keeps them so). Per rank, an exact integer checksum of each stage's flat parameters it holds (the fp32 bit
    patterns summed as int64, plus a position-weighted sum); MIN and MAX over ranks must agree for every stage.
    SDML_BENCH_PERTURB_RANK=k (tests only) flips one parameter bit on rank k first, so the check must fail."""
    P = engine.P
    big, small = 2 ** 62, -(2 ** 62)
    lo = torch.full((2 * P,), big, dtype=torch.int64)
    hi = torch.full((2 * P,), small, dtype=torch.int64)
    perturb = os.environ.get("SDML_BENCH_PERTURB_RANK")
    for s, mod in engine.stages.items():
        flat = torch.cat([p.detach().reshape(-1).float() for p in mod.parameters()])
        if perturb is not None and int(perturb) == rank:
            flat = flat.clone()
            flat[0] = torch.nextafter(flat[0], torch.tensor(float("inf"), device=flat.device))
        bits = flat.contiguous().view(torch.int32).to(torch.int64).cpu()
        w = torch.arange(1, bits.numel() + 1, dtype=torch.int64) % 65521
        c = torch.stack([bits.sum(), (bits * w).sum()])
        lo[2 * s:2 * s + 2] = c
        hi[2 * s:2 * s + 2] = c
    t_lo, t_hi = lo.to(dev), hi.to(dev)
    if mesh.backend == "gloo":
        t_lo, t_hi = lo, hi
    dist.all_reduce(t_lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(t_hi, op=dist.ReduceOp.MAX)
    lo, hi = t_lo.cpu(), t_hi.cpu()
    held = [s for s in range(P) if int(lo[2 * s]) != big]
    same = all(int(lo[2 * s + j]) == int(hi[2 * s + j]) for s in held for j in range(2))
    return {"identical": bool(same), "stages_checked": held,
            "checksums": {str(s): [int(lo[2 * s]), int(lo[2 * s + 1])] for s in held}}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(_launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        # a mislabelled run (e.g. --gpus 8 on a 1-rank launch) would report a flat scaling curve
        if rank == 0:
            print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={world}: refusing to run", file=sys.stderr)
        sys.exit(2)
    n = world
    place = a.placement
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    link_meas, link = None, plc.LinkModel()
    if n > 1 and a.link_probe != "off":
        # join the default process group first (init_mesh below reuses it) and measure the links the placements use
        from simple_distributed_machine_learning_amd.parallel import linkprobe

        m0 = init_mesh(pp=1, schedule_kind="rotate", timeout_s=900, rank=rank, world_size=world, p2p_channels=False)
        pdev = m0.device if m0.backend == "nccl" else torch.device("cpu")
        try:
            link_meas = linkprobe.measure(pdev, boundary_bytes=a.batch_per_gpu * (512 + 40))
            link = linkprobe.link_model(link_meas)
            link.allreduce_us = link_meas["allreduce_us"]
        except Exception as e:  # noqa: BLE001 - the assumed constants stand in (recorded in the JSON)
            link_meas = {"error": f"{type(e).__name__}: {e}"[:300]}
    rccl_world = n > 1 and os.environ.get("SDML_TRANSPORT", "direct") == "direct" and torch.cuda.device_count() > 0
    graph_dp = rccl_world and a.graph != "off" and not plc.dp_split_default()
    predicted = plc.table(n, a.batch_per_gpu, link=link, graph_dp=graph_dp if n > 1 else None)
    phi = None
    if n == 1:
        place = "dp"
    elif place == "auto":
        place, phi, _ = plc.choose(n, a.batch_per_gpu, link=link, graph_dp=graph_dp)
    if a.schedule is not None and n > 1:
        place = "pp2dp"
    if place == "pp2dp" and n % 2:
        raise SystemExit(f"pp2dp needs an even number of GPUs, got {n}")
    if place == "pp2dp":
        kind = a.schedule or "chimera"
        pp = 2
        M = a.microbatches or 4
        B = a.batch_per_gpu * pp  # per pipeline replica
        phi = 1.0
    else:
        kind = "rotate"
        pp = world
        if place == "dp":
            phi = 0.0
        elif place == "balanced":
            phi = plc.balanced_fraction(n, a.batch_per_gpu, link)
        elif place == "rotate":
            phi = None
        if a.cross_fraction is not None:
            phi = a.cross_fraction
        W = a.waves or (1 if (n == 1 or phi == 0) else 2)
        M = W * pp
        B = a.batch_per_gpu  # per owner shard
    # rotate on a 2-stage model runs its boundary as all-to-all collectives: no p2p channels
    mesh = init_mesh(pp=pp, schedule_kind=kind, timeout_s=900, rank=rank, world_size=world,
                     p2p_channels=(kind != "rotate"))
    dev = mesh.device
    knobs = {}
    if dev.type == "cuda":
        from simple_distributed_machine_learning_amd import _native

        knobs = _native.apply_knobs_from_env()  # A/B runs only (SDML_KNOBS="NAME=V,..."); default: none
    spec = get_model_spec(a.model, 2)
    engine = PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.1, momentum=0.5, seed=1,
                            cross_fraction=phi if kind == "rotate" else None)
    engine.train()
    GB = B * engine.data_shards  # samples per optimizer step, whole node
    # fresh data every step, cycling over `dataset_batches` global batches; a rank
    # materialises images only for the shards it feeds into stage 0 (labels for all)
    if world == 1:
        ds = SyntheticMNIST(GB * a.dataset_batches, seed=1234, device=dev, pixels=a.pixels)
    else:  # rotate: own shard of the group block; chimera/1f1b: the replica's whole batch
        own_lo = engine.local_start(0, B) + (mesh.pp_rank * B if kind == "rotate" else 0)
        ds = _ShardedSynth(GB, own_lo, B, a.dataset_batches, dev, pixels=a.pixels)

    # A graph replay is one host call for the whole step (full forward + backward + all-reduce + SGD, same kernels).
    # N > 1, dp over RCCL: the eager step waits ~25 us on the device between the gradient reduction and the optimizer
    # launch (the cross-stream hand-offs to and from the collective's stream); replayed, those are graph edges and the
    # step runs within ~3.5 us of the one-GPU step (profiles/r5_dp_graph_one_rank_rccl.jsonl). N = 1 has no collective,
    # and there the replayed kernels ran ~4 us per step slower than eager launches (profiles/r5_ab_graph_replay.jsonl).
    rccl = engine.transport is not None and engine.transport.name == "direct"
    use_graph = dev.type == "cuda" and (a.graph == "on" or (
        a.graph == "auto" and world > 1 and place == "dp" and rccl and not engine.dp_split))
    graphed = None
    nbatches = a.dataset_batches
    if use_graph:
        # one graph per cycled batch, captured on its first visit (the first step runs eagerly): cycle over at most
        # warmup - 1 batches so every capture happens during warm-up, none inside the timed region
        nbatches = max(1, min(a.dataset_batches, a.warmup - 1))
        from simple_distributed_machine_learning_amd.parallel.graphs import GraphedStep

        graphed = GraphedStep(engine, allow_collectives=world > 1, direct_data=True,
                              max_direct=max(1, a.dataset_batches))

    def step(i):
        start = (i % nbatches) * GB
        if graphed is not None:
            return graphed(ds, engine.local_start(start, B), B, global_batch=GB)
        return engine.run(ds, engine.local_start(start, B), B, train=True, global_batch=GB)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        mesh.barrier()

    for i in range(a.warmup):
        step(i)
    graphs_before_timing = len(graphed.graphs) if graphed is not None else 0
    if graphed is not None and world > 1:
        # every rank replays or none does (a capture that failed on one rank leaves that rank eager; the collective
        # sequence would still match, but the timed steps should run one code path everywhere)
        ok = torch.tensor([0.0 if graphed.disabled else 1.0], device=dev)
        engine.transport.all_reduce(ok, channel="world", op=dist.ReduceOp.MIN, async_op=False)
        if float(ok.item()) < 1.0:
            graphed.disabled = True
    sync()
    if engine.transport is not None:
        engine.transport.reset_counters()
    # per-step device time: one event before every timed step and one after the last, recorded on the
    # compute stream (host cost ~1 us each); read after the timed region. They describe the window the
    # wall clock measures (first step vs steady state), they do not replace it.
    # SDML_BENCH_EVENTS (A/B): "all" = an event before every step, "ends" = around the first step and at the end only,
    # "none"
    # (measured, profiles/r6_bench_events_ab.jsonl: an event before every step costs ~4.5 us of device time per step -
    # a marker between two kernels of one stream stops the next dispatch from overlapping the previous one's tail)
    ev_mode = os.environ.get("SDML_BENCH_EVENTS", "ends") if dev.type == "cuda" else "none"
    rec = set(range(a.steps + 1)) if ev_mode == "all" else ({0, 1, a.steps} if ev_mode == "ends" else set())
    evs = {i: torch.cuda.Event(enable_timing=True) for i in rec}
    t0 = time.perf_counter()
    res = None
    for i in range(a.steps):
        if i in evs:
            evs[i].record()
        res = step(a.warmup + i)
    if a.steps in evs:
        evs[a.steps].record()
    sync()
    el = time.perf_counter() - t0
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)] if ev_mode == "all" else []
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    sent = torch.tensor([float(engine.transport.bytes_sent if engine.transport else 0)], dtype=torch.float64,
                        device=dev)
    if world > 1:
        engine.transport.all_reduce(t, channel="world", op=dist.ReduceOp.MAX, async_op=False)
        engine.transport.all_reduce(sent, channel="world", async_op=False)
    el = float(t.item())
    cross_bytes = float(sent.item()) / a.steps
    replicas = _replica_check(engine, mesh, dev, rank) if world > 1 else None
    loss = None
    if res is not None:
        l, c, cnt = engine.reduce_metrics(res)
        loss = l / max(1, cnt)
    sps = GB * a.steps / el
    # the reference's own placement, measured next to the chosen one (after the timed region)
    alternatives = {}
    want_alt = a.alternatives == "on" or (a.alternatives == "auto" and n % 2 == 0)
    if want_alt and n > 1 and n % 2 == 0 and place != "pp2dp" and a.model == "mlp":
        try:
            alternatives["pp2dp"] = _measure_pp2dp(a, n, rank, world, dev)
        except Exception as e:  # noqa: BLE001 - the headline number above stands on its own
            alternatives["pp2dp"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    # what the process group really saw (1 and None for a single-GPU run without collectives)
    seen_world = dist.get_world_size() if dist.is_initialized() else 1
    seen_backend = dist.get_backend() if dist.is_initialized() else None
    if seen_world != n:
        raise SystemExit(f"[bench] process group has {seen_world} ranks, expected {n}")
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
                "parallelism": _parallelism(place, n, mesh, phi, kind),
                "placement": place,
                "cross_fraction": phi if place != "rotate" else round((n - 1) / n, 4),
                "boundary_bytes_across_gpus_per_step": int(cross_bytes),
                "transport": engine.transport.name if engine.transport else None,
                "world_size_seen": seen_world,
                "backend": seen_backend,
                "link_model": plc.model_dict(link),
                "link_model_assumed": plc.model_dict()["link"],
                "link_measured": link_meas,
                "replicas_identical": None if replicas is None else replicas["identical"],
                "replica_check": replicas,
                "predicted": predicted,
                "measured_alternatives": alternatives,
                "kernel_knobs": knobs,
                "hip_graph": None if graphed is None else {"graphs": len(graphed.graphs), "replays": graphed.replays,
                                                           "eager_steps": graphed.eager_steps,
                                                           "disabled": graphed.disabled,
                                                           "captures_in_timed_region":
                                                               len(graphed.graphs) - graphs_before_timing,
                                                           "dataset_batches_cycled": nbatches},
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
        if ev_mode == "ends" and a.steps >= 2:
            out["step_ms_events"] = {"first": round(evs[0].elapsed_time(evs[1]), 4),
                                     "rest_mean": round(evs[1].elapsed_time(evs[a.steps]) / (a.steps - 1), 4)}
        if step_ms:  # rank 0's per-step device times (HIP events on the compute stream)
            srt = sorted(step_ms)
            out["step_ms_events"] = {"first": round(step_ms[0], 4), "median": round(srt[len(srt) // 2], 4),
                                     "min": round(srt[0], 4), "max": round(srt[-1], 4),
                                     "all": [round(x, 4) for x in step_ms]}
        print(json.dumps(out), flush=True)
    if world > 1:
        sync()
        dist.destroy_process_group()
    if replicas is not None and not replicas["identical"]:
        if rank == 0:
            print("[bench] replicas diverged: " + json.dumps(replicas), file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
