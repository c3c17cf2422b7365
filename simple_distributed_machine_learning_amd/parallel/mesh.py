"""Process-group bootstrap and the dp x pp rank mesh.

Replaces the reference's RPC bootstrap (``rpc.init_rpc`` / ``rpc.shutdown``,
/root/reference/simple_distributed.py:167-186): instead of a "master" that drives remote
modules, every rank joins ONE ``torch.distributed`` process group (RCCL — PyTorch-ROCm's
``"nccl"`` backend — on MI355X, Gloo on the CPU test path) and runs the same SPMD program.

Rank layout: ``rank = (dp_rank * pp + pp_rank) * tp + tp_rank`` — the tensor-parallel ranks of
a stage (parallel/tp.py) are adjacent, then the stages of one pipeline, then the replicas. On an
8-GPU node the stage pairs (0,1), (2,3), ... (tp = 1) each talk over their own direct xGMI link
and DP replicas of a stage all-reduce over the other links. A pipeline's stage-to-stage
messages go between ranks with the same ``tp_rank``.

Point-to-point traffic uses one 2-rank process group per *ordered* neighbour pair
(direction). Each group owns its own RCCL communicator and HIP stream, so every
direction is an independent FIFO channel — exactly the model the native schedule
validator (csrc/runtime/schedule.cpp) proves deadlock-free.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass
class Mesh:
    rank: int
    world_size: int
    local_rank: int
    pp: int  # ranks per pipeline
    dp: int  # pipeline replicas
    schedule_kind: str
    device: torch.device
    backend: str
    pp_rank: int = 0
    dp_rank: int = 0
    # (src_global, dst_global) -> group carrying src->dst messages
    p2p_groups: Dict[Tuple[int, int], object] = field(default_factory=dict)
    # group used to all-reduce this rank's gradients (None: nothing to reduce)
    grad_group: Optional[object] = None
    grad_group_ranks: List[int] = field(default_factory=list)
    pipe_group: Optional[object] = None
    initialized_here: bool = False
    tp: int = 1  # tensor-parallel ranks per stage
    tp_rank: int = 0
    tp_group: Optional[object] = None
    # rotate: a second communicator over the pipeline ranks for the backward boundary exchange, so
    # it does not queue behind the next wave's forward exchange on one RCCL stream
    pipe_group_bwd: Optional[object] = None
    # how cross-rank bytes move (parallel/p2p.py): "direct" = torch.distributed on the tensors
    # themselves (RCCL for device tensors, Gloo for CPU ones); "host" = device tensors staged
    # through host memory over Gloo (several ranks sharing one GPU)
    transport_kind: str = "direct"
    _transport: Optional[object] = None

    # a one-rank mesh that still builds its communicators and runs its collectives (graph-capture
    # and RCCL checks on one GPU: init_mesh(force_collectives=True) inside a 1-rank process group)
    force_collectives: bool = False

    @property
    def transport(self):
        """The rank's :class:`~.p2p.Transport` (None on a 1-rank mesh)."""
        if self.world_size == 1 and not self.force_collectives:
            return None
        if self._transport is None:
            from .p2p import make_transport

            self._transport = make_transport(self)
        return self._transport

    def barrier(self):
        if self.world_size > 1:
            self.transport.barrier()

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    def global_rank(self, dp_rank: int, pp_rank: int) -> int:
        """Global rank of pipeline position (dp_rank, pp_rank) in THIS rank's tensor-parallel slice."""
        return (dp_rank * self.pp + pp_rank) * self.tp + self.tp_rank

    def tp_context(self):
        from .tp import TPContext

        return TPContext(self.tp, self.tp_rank, self.tp_group, self.transport)

    def pipe_ranks(self) -> List[int]:  # this rank's pipeline (same dp_rank, same tp_rank)
        return [self.global_rank(self.dp_rank, r) for r in range(self.pp)]

    def is_master(self) -> bool:
        return self.rank == 0


def select_device(local_rank: int) -> torch.device:
    if torch.cuda.is_available():
        n = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(n, 1))
        torch.cuda.set_device(dev)
        return dev
    return torch.device("cpu")


def default_backend(device: torch.device) -> str:
    # "nccl" is RCCL on PyTorch-ROCm: the collective/p2p library over xGMI.
    return "nccl" if device.type == "cuda" else "gloo"


def replica_groups_spec(world_size: int, pp: int, kind: str, tp: int = 1) -> List[List[int]]:
    """Lists of ranks that hold replicas of the same parameters (gradient all-reduce groups):
    the same stage set at the same tensor-parallel position."""
    dp = world_size // (pp * tp)
    groups = []
    if kind == "rotate":  # every rank hosts every stage: one group over the whole world
        return [list(range(world_size))]
    for t in range(tp):
        seen = set()
        for r in range(pp):
            mirror = pp - 1 - r if kind == "chimera" else r
            key = tuple(sorted({r, mirror}))
            if key in seen:
                continue
            seen.add(key)
            ranks = sorted((d * pp + x) * tp + t for d in range(dp) for x in key)
            groups.append(ranks)
    return groups


def _pg_options(backend: str):
    """RCCL groups get a HIGH-priority communication stream (SDML_COMM_HIGH_PRIO=0 turns it off).

    The bf16x3 GEMMs occupy a whole CU each (144 KiB LDS, 2 x ~250 VGPRs per SIMD), so an RCCL
    kernel launched beside them cannot start until CUs free up; at equal priority the next
    compute kernel competes for those CUs. A high-priority stream lets the boundary all-to-all and
    the gradient all-reduce take CUs first, so they overlap the following compute."""
    if backend != "nccl" or os.environ.get("SDML_COMM_HIGH_PRIO", "1") == "0":
        return None
    try:
        o = dist.ProcessGroupNCCL.Options()
        o.is_high_priority_stream = True
        return o
    except Exception:  # noqa: BLE001 - an optimisation only
        return None


def init_mesh(pp: int, schedule_kind: str = "1f1b", backend: Optional[str] = None,
              timeout_s: float = 600.0, rank: Optional[int] = None, world_size: Optional[int] = None,
              local_rank: Optional[int] = None, device: Optional[torch.device] = None,
              p2p_channels: bool = True, tp: int = 1, transport: Optional[str] = None,
              force_collectives: bool = False) -> Mesh:
    """Join (or reuse) the default process group and build the dp x pp mesh.

    Rank/world come from arguments, else torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK).
    ``MASTER_ADDR``/``MASTER_PORT`` must be set for world_size > 1 (TCPStore rendezvous, the
    same store the reference's ``init_rpc`` used). The timeout is finite:
    the reference's ``rpc_timeout=0`` means "wait forever" and, on torch 2.10, an instant
    rendezvous failure.

    ``transport`` (default: env ``SDML_TRANSPORT``, else ``"direct"``): ``"host"`` stages device
    tensors through host memory over Gloo, so several ranks can share one GPU (RCCL refuses
    that); the process group is then Gloo even on a ROCm device. ``"ipc"`` moves the
    point-to-point boundary tensors device to device through hipIPC (parallel/p2p.py
    IpcTransport; same GPU or peers), its collectives host-staged over the Gloo group.
    """
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        device = select_device(local_rank)
    transport = transport or os.environ.get("SDML_TRANSPORT", "direct")
    if transport not in ("direct", "host", "ipc"):
        raise ValueError(f"unknown transport {transport!r} (direct | host | ipc)")
    if transport == "ipc" and device.type != "cuda":
        transport = "direct"  # (no device: the CPU test path has nothing to map)
    if backend is None:
        backend = "gloo" if transport in ("host", "ipc") else default_backend(device)
    if backend == "gloo" and device.type == "cuda" and transport != "ipc":
        transport = "host"  # Gloo cannot run the engine's collectives on device tensors
    tp = max(1, int(tp))
    if world_size % tp != 0:
        raise ValueError(f"world_size={world_size} is not a multiple of tensor-parallel ranks tp={tp}")
    if tp > 1 and schedule_kind in ("rotate", "chimera"):
        raise ValueError(f"tensor parallelism runs with the gpipe / 1f1b schedules, not {schedule_kind!r}")
    pp = max(1, min(pp, world_size // tp))
    if world_size % (pp * tp) != 0:
        raise ValueError(f"world_size={world_size} is not a multiple of pp={pp} x tp={tp}")
    mesh = Mesh(rank=rank, world_size=world_size, local_rank=local_rank, pp=pp, dp=world_size // (pp * tp),
                schedule_kind=schedule_kind, device=device, backend=backend, tp=tp, transport_kind=transport)
    mesh.tp_rank = rank % tp
    mesh.pp_rank = (rank // tp) % pp
    mesh.dp_rank = rank // (tp * pp)
    mesh.force_collectives = bool(force_collectives and world_size == 1 and dist.is_initialized())
    if world_size == 1 and not mesh.force_collectives:
        return mesh

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kwargs = dict(backend=backend, rank=rank, world_size=world_size,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = device
            opts = _pg_options(backend)
            if opts is not None:
                kwargs["pg_options"] = opts
        dist.init_process_group(**kwargs)
        mesh.initialized_here = True

    # ---- groups: every rank creates every group in the same order (collective) ----
    timeout = datetime.timedelta(seconds=timeout_s)
    opts = _pg_options(backend)

    def new_group(ranks):
        return dist.new_group(ranks, timeout=timeout, pg_options=opts)

    for d in range(mesh.dp):
        for t in range(tp):
            ranks = [(d * pp + r) * tp + t for r in range(pp)]
            g = new_group(ranks) if pp > 1 else None
            gb = new_group(ranks) if pp > 1 and schedule_kind == "rotate" else None
            if d == mesh.dp_rank and t == mesh.tp_rank:
                mesh.pipe_group = g
                mesh.pipe_group_bwd = gb
    # rotate talks to every peer of the pipeline group; the others only to neighbours
    pairs = [(r, q) for r in range(pp) for q in range(r + 1, pp)] if schedule_kind == "rotate" else \
        [(r, r + 1) for r in range(pp - 1)]
    if not p2p_channels:
        pairs = []
    for d in range(mesh.dp):
        for t in range(tp):
            for r, q in pairs:
                a, b = (d * pp + r) * tp + t, (d * pp + q) * tp + t
                for src, dst in ((a, b), (b, a)):
                    g = new_group([a, b])
                    if mesh.rank in (a, b):
                        mesh.p2p_groups[(src, dst)] = g
    for ranks in replica_groups_spec(world_size, pp, schedule_kind, tp):
        real = len(ranks) > 1 or mesh.force_collectives
        g = new_group(ranks) if real else None
        if rank in ranks and real:
            mesh.grad_group = g
            mesh.grad_group_ranks = ranks
    if tp > 1:
        for d in range(mesh.dp):
            for r in range(pp):
                ranks = [(d * pp + r) * tp + t for t in range(tp)]
                g = new_group(ranks)
                if rank in ranks:
                    mesh.tp_group = g
    return mesh


def shutdown(mesh: Optional[Mesh] = None):
    """Graceful teardown: barrier then destroy (the reference's ``rpc.shutdown()`` also
    blocks until every rank arrives, simple_distributed.py:186)."""
    if dist.is_initialized():
        try:
            if mesh is not None and mesh.world_size > 1:
                mesh.barrier()
            else:
                dist.barrier()
        finally:
            dist.destroy_process_group()
