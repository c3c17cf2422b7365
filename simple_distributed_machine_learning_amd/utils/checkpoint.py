"""Per-stage checkpoint / resume.

The reference never checkpoints. Its only persistent "layout" is the module
attribute names of each stage (conv1.*, conv2.* on stage 0; fc1.*, fc2.* on stage 1), which
these files keep verbatim:

    <dir>/stage{k}.pt = {"model": state_dict (reference key names),
                         "optim": {"momentum_buffer": {name: tensor}, "steps": n, ...},
                         "epoch", "batch", "global_step", "stage", "num_stages", "model_name"}
    <dir>/rng_rank{r}.pt = per-rank RNG states (bit-identical resume of dropout)
    with tensor parallelism (tp > 1) every tp rank writes its shard: stage{k}_tp{t}.pt

Exactly one rank writes each stage file (the dp-rank-0 holder of the stage in pipe 0); all
holders of a stage (DP replicas, Chimera mirrors) load the same file. Loading uses
``torch.load(weights_only=True)``: nothing in the file is executed.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Optional

import torch

from ..parallel.pipeline import PipelineEngine


def _atomic_save(obj, path: Path):
    tmp = path.with_name(path.name + ".tmp")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _stage_file(d: Path, s: int, mesh) -> Path:
    return d / (f"stage{s}.pt" if mesh.tp == 1 else f"stage{s}_tp{mesh.tp_rank}.pt")


def save_checkpoint(engine: PipelineEngine, ckpt_dir: str, epoch: int, batch: int, extra: Optional[dict] = None):
    d = Path(ckpt_dir)
    d.mkdir(parents=True, exist_ok=True)
    sched = engine.schedule(engine.M, False)
    mesh = engine.mesh
    for s, mod in engine.stages.items():
        writer = mesh.dp_rank == 0 and sched.stage_rank(0, s) == mesh.pp_rank
        if not writer:
            continue
        sd = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
        obj = {"model": sd, "optim": engine.optimizer.state_dict_for_stage(s), "epoch": int(epoch),
               "batch": int(batch), "global_step": int(engine.global_step), "stage": int(s),
               "num_stages": int(engine.P), "model_name": engine.spec.name}
        if extra:
            obj.update(extra)
        if mesh.tp > 1:
            obj["tp"], obj["tp_rank"] = int(mesh.tp), int(mesh.tp_rank)
        _atomic_save(obj, _stage_file(d, s, mesh))
    rng = {"cpu": torch.get_rng_state(), "step_ctr": engine.step_ctr.detach().cpu()}
    if engine.device.type == "cuda":
        rng["cuda"] = torch.cuda.get_rng_state(engine.device)
    _atomic_save(rng, d / f"rng_rank{mesh.rank}.pt")


def load_checkpoint(engine: PipelineEngine, ckpt_dir: str, strict: bool = True) -> dict:
    """Load every local stage; returns {"epoch", "batch", "global_step"} of the checkpoint."""
    d = Path(ckpt_dir)
    meta = {"epoch": 0, "batch": -1, "global_step": 0}
    for s, mod in engine.stages.items():
        path = _stage_file(d, s, engine.mesh)
        obj = torch.load(path, map_location="cpu", weights_only=True)
        if int(obj.get("tp", 1)) != engine.mesh.tp:
            raise ValueError(f"{path}: saved with tp={obj.get('tp', 1)}, running with tp={engine.mesh.tp}")
        if obj.get("model_name") not in (None, engine.spec.name):
            raise ValueError(f"{path}: checkpoint is for model {obj.get('model_name')!r}, not {engine.spec.name!r}")
        with torch.no_grad():
            missing, unexpected = mod.load_state_dict(obj["model"], strict=strict)
        engine.optimizer.load_state_dict_for_stage(s, obj.get("optim", {}))
        meta = {"epoch": int(obj.get("epoch", 0)), "batch": int(obj.get("batch", -1)),
                "global_step": int(obj.get("global_step", 0))}
    rng_path = d / f"rng_rank{engine.mesh.rank}.pt"
    if rng_path.exists():
        rng = torch.load(rng_path, map_location="cpu", weights_only=True)
        torch.set_rng_state(rng["cpu"])
        if "cuda" in rng and engine.device.type == "cuda":
            torch.cuda.set_rng_state(rng["cuda"], engine.device)
        if "step_ctr" in rng:
            engine.step_ctr.copy_(rng["step_ctr"])
    engine.global_step = meta["global_step"]
    return meta
