"""Rank bodies for the multi-process tests (module-level so spawn can import them)."""
from __future__ import annotations

import torch


def train_worker(rank, world, model, kind, M, pp, steps, B, seed=3, kw=None, tp=1):
    from simple_distributed_machine_learning_amd.data import SyntheticMNIST, SyntheticTokens
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    kw = dict(kw or {})
    # engine/mesh options (not model options): device ("cpu" | "cuda"), transport, cross_fraction
    dev = torch.device(kw.pop("device", "cpu"))
    transport = kw.pop("transport", None)
    eng_kw = {k: kw.pop(k) for k in ("cross_fraction",) if k in kw}
    dp_split = kw.pop("dp_split", False)
    mesh = init_mesh(pp=pp, schedule_kind=kind, rank=rank, world_size=world, device=dev,
                     backend="gloo", timeout_s=120, tp=tp, transport=transport)
    spec = get_model_spec(model, kw.get("stages"), **{k: v for k, v in kw.items() if k not in ("stages", "pixels")})
    eng = PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.1, momentum=0.5, seed=seed,
                         **eng_kw)
    if dp_split:
        eng.dp_split = True
    S = eng.data_shards
    if spec.input_kind == "tokens":
        ds = SyntheticTokens(B * S * steps, kw.get("seq_len", 16), 97, seed=7, device=dev)
    else:
        ds = SyntheticMNIST(B * S * steps, seed=7, pixels=kw.get("pixels", "f32"), device=dev)
    losses = []
    allocs_first = None
    for step in range(steps):
        if step == 1:
            allocs_first = eng.bufs.allocations
        res = eng.run(ds, eng.local_start(step * B * S, B), B, train=True, global_batch=B * S)
        l, c, n = eng.reduce_metrics(res)
        losses.append(l / n)
    # one forward-only pass (eval schedule)
    eng.eval()
    res = eng.run(ds, eng.local_start(0, B), B, train=False)
    el, ec, en = eng.reduce_metrics(res)
    return {"losses": losses, "state": eng.state_dicts(), "dp_rank": mesh.dp_rank, "pp_rank": mesh.pp_rank,
            "tp_rank": mesh.tp_rank,
            "eval": (el, ec, en), "bytes_sent": eng.transport.bytes_sent if eng.transport else 0,
            "transport": eng.transport.name if eng.transport else None,
            "pool_allocs": eng.bufs.allocations, "pool_allocs_first": allocs_first,
            "dp_split_steps": eng.dp_split_steps}


def empty_replica_worker(rank, world, pp, B, steps, seed=3, dp_split=False, cross_fraction=None):
    """rotate, dp replicas of a pp-rank group: replica 1 gets NO samples every step (batch 0), replica 0
    gets B per owner; global_batch is fixed to replica 0's samples. Returns the trained weights.
    ``dp_split``: the split gradient all-reduce is planned (two spans per step on every replica)."""
    from simple_distributed_machine_learning_amd.data import SyntheticMNIST
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    mesh = init_mesh(pp=pp, schedule_kind="rotate", rank=rank, world_size=world, device=torch.device("cpu"),
                     backend="gloo", timeout_s=120)
    eng = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=2 * pp, lr=0.1,
                         momentum=0.5, seed=seed, cross_fraction=cross_fraction)
    eng.dp_split = dp_split
    spans = []
    real_issue = eng.grad_sync.issue_span
    eng.grad_sync.issue_span = lambda lo, hi: (spans.append((lo, hi)), real_issue(lo, hi))
    ds = SyntheticMNIST(B * pp * steps, seed=7)
    for step in range(steps):
        n = B if mesh.dp_rank == 0 else 0
        eng.run(ds, step * B * pp, n, train=True, global_batch=B * pp)
    return {"state": eng.state_dicts(), "dp_rank": mesh.dp_rank, "spans": spans}


def debug_sync_rotate_worker(rank, world, B):
    """rotate, debug_sync: a bad label in a PEER's shard (rows every head may see) must be refused on every
    rank before any collective. Returns the error text (None if nothing was raised)."""
    from simple_distributed_machine_learning_amd.data import SyntheticMNIST
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    mesh = init_mesh(pp=world, schedule_kind="rotate", rank=rank, world_size=world, device=torch.device("cpu"),
                     backend="gloo", timeout_s=60)
    eng = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=2 * world,
                         lr=0.1, momentum=0.5, seed=1, debug_sync=True)
    ds = SyntheticMNIST(B * world, seed=7)
    ds.y[(world - 1) * B + 3] = 10  # owned by the last rank
    try:
        eng.run(ds, 0, B, train=True)
    except ValueError as e:
        return str(e)
    return None
