"""SPMD pipeline engine: executes a validated schedule on one rank.

What it replaces in the reference (/root/reference/simple_distributed.py):

=====================================  ==================================================
reference                              here
=====================================  ==================================================
``rpc.remote('worker1', Network2)``    every rank builds the stages it owns (:meth:`__init__`)
(:33-37)
``RRef(z3)`` + ``rpc_sync().forward``  ``isend`` of the boundary activation to the next
+ ``to_here()`` (:47-49, :71)          rank, ``irecv`` into a fresh buffer there
``dist_autograd.context/backward``     explicit per-stage backward seeded by the received
(:109-112)                             gradient; input-grad sent to the previous rank
``DistributedOptimizer.step`` (:113)   one fused SGD launch over the rank's flat buffer
``nll_loss`` on the master (:111)      loss on the LAST stage; labels read locally
=====================================  ==================================================

Within a step nothing blocks the host except optional metric reads: receives are
stream-level waits, sends are drained at the end of the step, and the data-parallel
gradient all-reduce for a stage is issued as soon as that stage's last backward is done
(overlapping the remaining backward work of other stages on the rank).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..models.base import ModelSpec, PipelineStage, build_stages
from .. import ops
from ..ops import pixels_to_float
from ..ops.side_stream import join_side_streams
from ..ops.optim import FusedSGD
from ..utils.flat import FlatParams
from ..utils.timing import PhaseTimer
from .mesh import Mesh
from .p2p import BufferPool, message_tag
from .schedule import OP_BWD, OP_FWD, OP_RECV, OP_SEND, PL_ACT, PL_GRAD, Schedule, build_schedule


def split_sizes(n: int, m: int) -> List[int]:
    """Micro-batch sizes (torch.tensor_split convention): first ``n % m`` get one more."""
    m = max(1, min(m, n))
    base, extra = divmod(n, m)
    return [base + (1 if i < extra else 0) for i in range(m)]


@dataclass
class StepResult:
    loss_sum: torch.Tensor  # 0-dim, summed over the samples this rank's last stage(s) saw
    correct: torch.Tensor   # 0-dim (float32 count)
    count: int
    wall_s: float = 0.0

    def mean_loss(self) -> float:
        return float(self.loss_sum) / max(1, self.count)


class GradSync:
    """Data-parallel / Chimera-mirror gradient all-reduce over the flat grad buffer.

    Stages are reduced in a canonical order (descending stage id) so every member of the
    replica group issues the same collective sequence; a stage's all-reduce is launched as
    soon as it and all stages before it in that order have finished backward.
    """

    def __init__(self, flat: FlatParams, mesh: Mesh, local_stages: Sequence[int]):
        self.flat, self.mesh = flat, mesh
        self.transport = mesh.transport
        self.order = sorted(set(local_stages), reverse=True)
        self.enabled = mesh.grad_group is not None
        self._done = set()
        self._ptr = 0
        self._works = []
        self._span_hi = 0  # issue_span: gradient prefix [0, _span_hi) already handed to all-reduces
        # merge consecutive stages into one contiguous bucket when they are adjacent in memory
        self.group = mesh.grad_group

    def reset(self):
        self._done.clear()
        self._ptr = 0
        self._works = []
        self._span_hi = 0

    def stage_done(self, stage: int):
        if not self.enabled:
            return
        self._done.add(stage)
        while self._ptr < len(self.order) and self.order[self._ptr] in self._done:
            s = self.order[self._ptr]
            t = self.flat.stage_slice(s, "grads")
            self._works.append(self.transport.all_reduce(t, channel="grad"))
            self._ptr += 1

    def issue_span(self, lo: int, hi: int):
        """All-reduce ``flat.grads[lo:hi]`` now: a finished, contiguous range of the gradient whose
        collective then runs (RCCL stream) under the kernels that still compute the rest. Spans are issued
        in buffer order and must end up covering the whole buffer (checked by :meth:`finish_all`)."""
        if not self.enabled:
            return
        if lo != self._span_hi or hi <= lo or hi > self.flat.grads.numel():
            raise RuntimeError(f"GradSync.issue_span [{lo}, {hi}) does not continue [0, {self._span_hi})")
        self._works.append(self.transport.all_reduce(self.flat.grads[lo:hi], channel="grad"))
        self._span_hi = hi

    def finish_all(self):
        """ONE all-reduce over the whole flat gradient buffer (every local stage at once): fewer
        collectives when nothing is left to overlap them with (rotate / dp placements). After
        :meth:`issue_span` calls it waits for those instead (every rank issues the same spans)."""
        if not self.enabled:
            return
        if self._ptr:
            raise RuntimeError("GradSync.finish_all after per-stage all-reduces were issued")
        if self._works:
            if self._span_hi != self.flat.grads.numel():
                raise RuntimeError("GradSync.finish_all: the issued spans do not cover the gradient")
            for w in self._works:
                w.wait()
            self._works = []
            self._span_hi = 0
            return
        self.transport.all_reduce(self.flat.grads, channel="grad").wait()

    def finish(self):
        if not self.enabled:
            return
        for s in self.order:
            self.stage_done(s)
        for w in self._works:
            w.wait()
        self._works = []


class PipelineEngine:
    def __init__(self, spec: ModelSpec, mesh: Mesh, schedule_kind: str = "1f1b", num_microbatches: int = 1,
                 lr: float = 0.1, momentum: float = 0.5, weight_decay: float = 0.0, seed: int = 0,
                 dtype: Optional[torch.dtype] = None, debug_sync: bool = False, timing: bool = False,
                 cross_fraction: Optional[float] = None):
        self.spec, self.mesh = spec, mesh
        self.kind = schedule_kind
        self.M = max(1, int(num_microbatches))
        self.P = spec.num_stages
        if schedule_kind != "rotate" and self.P % mesh.pp != 0:
            raise ValueError(f"{spec.name}: {self.P} stages cannot be placed on {mesh.pp} pipeline ranks")
        self.device = mesh.device
        self.dtype = dtype or spec.param_dtype
        self.debug_sync = debug_sync or os.environ.get("SDML_DEBUG_SYNC") == "1"
        self.timing = timing
        self.last_timing: Dict[str, float] = {}  # per-stage/phase ms of the last step (timing=True)
        self._sched_cache: Dict[Tuple[int, bool], Schedule] = {}
        if self.kind == "rotate" and self.M % mesh.pp:
            raise ValueError(f"rotate: micro-batches ({self.M}) must be a multiple of the ranks ({mesh.pp})")
        sched = self.schedule(self.M, False)
        self.local_pairs = sched.local_stages(mesh.pp_rank)
        if self.kind != "rotate":
            for p in range(sched.num_pipes):
                for s in range(self.P):
                    if sched.stage_rank(p, s) == mesh.pp_rank and (p, s) not in self.local_pairs:
                        self.local_pairs.append((p, s))
        self.local_stage_ids = sorted({s for _, s in self.local_pairs})
        mods = build_stages(spec, self.local_stage_ids, base_seed=seed)
        if mesh.tp > 1:  # tensor-parallel split of each local stage (parallel/tp.py)
            tpc = mesh.tp_context()
            for m in mods:
                if not getattr(m, "supports_tp", False):
                    raise ValueError(f"{spec.name} has no tensor-parallel implementation (tp={mesh.tp})")
                m.shard_tp(tpc)
        self.stages: Dict[int, PipelineStage] = {}
        for s, m in zip(self.local_stage_ids, mods):
            m.to(self.device)
            if self.dtype != torch.float32:
                m.to(self.dtype)
            self.stages[s] = m
        self.flat = FlatParams([(s, m) for s, m in self.stages.items()], self.device, self.dtype)
        # device-side training-step counter: fused dropout kernels mix it into their seeds, and
        # it is advanced by a (capturable) device op at the end of every training step, so a
        # replayed hipGraph draws fresh masks each step (see parallel/graphs.py)
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._uses_rng = False
        for m in self.stages.values():
            if getattr(m, "uses_rng_step", False):
                m.rng_step = self.step_ctr
                self._uses_rng = True
        self.optimizer = FusedSGD(self.flat, lr=lr, momentum=momentum, weight_decay=weight_decay)
        for m in self.stages.values():  # derived weight caches the step kernel keeps current
            if hasattr(m, "attach_plane_cache"):
                m.attach_plane_cache(self.flat, self.optimizer)
        # every cross-rank byte goes through the mesh's transport seam (parallel/p2p.py); boundary
        # buffers come from a persistent pool (no per-step communication allocations)
        self.transport = mesh.transport
        self.bufs = BufferPool(self.device)
        self.grad_sync = GradSync(self.flat, mesh, self.local_stage_ids)
        self.training = True
        self.global_step = 0
        # rotate, 2 stages: run each wave's stage boundary as ONE all-to-all collective
        # (RCCL drives all xGMI links at once; far fewer launches than per-peer p2p)
        self.use_alltoall = os.environ.get("SDML_ROTATE_P2P") != "1"
        # rotate all-to-all, 2-stage models with a single-Linear head: send the boundary gradient
        # as its rank-C factor (see _run_rotate_alltoall); SDML_ROTATE_FACTORED=0 sends it whole
        self.factored_boundary_grad = os.environ.get("SDML_ROTATE_FACTORED", "1") != "0"
        # ... also with both stages on one rank (R == 1): the head then skips its dx pass and stage 0
        # reads h + dl instead of dx (SDML_FACTORED_R1=0: the head returns dx)
        self.factored_r1 = os.environ.get("SDML_FACTORED_R1", "1") != "0"
        # rotate (2 stages): fraction of every wave whose stage 1 runs on a peer (rotate_parts);
        # None = classic equal shares. SDML_CROSS_FRACTION overrides.
        env_phi = os.environ.get("SDML_CROSS_FRACTION")
        if env_phi is not None:
            cross_fraction = float(env_phi)
        if cross_fraction is not None and not 0.0 <= cross_fraction <= 1.0:
            raise ValueError(f"cross_fraction must be in [0, 1], got {cross_fraction}")
        self.cross_fraction = cross_fraction
        # rotate: stage 0's forward and stage 1's forward+loss+backward in one kernel for the rows that
        # stay on their owner (models/mlp.py fwd_head_fused); SDML_FUSE_HEAD=0 keeps them separate
        self.fuse_head = os.environ.get("SDML_FUSE_HEAD", "1") != "0"
        # data-parallel gradient all-reduce overlapped with backward (rotate all-to-all, nothing crossing,
        # uint8 first layer): the first layer's weight gradient runs as two hidden-unit ranges, the first
        # range's rows are all-reduced while the second range's kernel runs (_dp_split_spans).
        # SDML_DP_SPLIT_BLOCKS: row splits per range (< 256 leaves CUs free for the RCCL kernel).
        # Opt-in (SDML_DP_SPLIT=1): measured on one MI355X (profiles/r4_dpsplit_one_rank_rccl*), the two
        # range launches cost 2 x 45 us against 77 us for the whole gradient (each range writes a full-size
        # partial slab: twice the slab traffic) plus a second reduction launch, +33 us per step in all,
        # more than the half all-reduce it can hide is expected to take at 8 ranks.
        self.dp_split = os.environ.get("SDML_DP_SPLIT", "0") == "1"
        self.dp_split_blocks = int(os.environ.get("SDML_DP_SPLIT_BLOCKS", "240"))
        self.dp_split_steps = 0  # training steps that ran the split (tests)
        self._small_step = None  # one-launch reference-size MLP step available (decided on first use)
        self._cnn_step = None  # two-launch reference CNN step available (decided on first use)
        self.fast_steps = {"mlp_small": 0, "cnn": 0}  # steps that ran the one/two-launch paths (tests)
        self._small_args = None
        self._cnn_args = None
        self._fuse_ok = {}  # _can_fuse_head memo
        self._wave_bufs = {}  # fused waves' persistent (ReLU bits, gradient) buffers
        # set by GraphedStep once a graph is captured: evicted wave buffers then stay alive (a graph holds their
        # addresses, not references), see _fused_wave_bufs and BufferPool.retain
        self.graph_retain = False
        self._wave_bufs_retired = []
        if self.kind == "rotate" and self.P == 2 and not self.use_alltoall and mesh.pp > 1 and not mesh.p2p_groups:
            raise ValueError("rotate with p2p transfers needs a mesh built with p2p_channels=True")

    def _advance_rng(self):
        if self._uses_rng:  # one tiny launch per step, only for models with fused dropout
            self.step_ctr.add_(1)

    # ---------------------------------------------------------------------------------------
    def schedule(self, m: int, forward_only: bool) -> Schedule:
        key = (m, forward_only)
        if key not in self._sched_cache:
            self._sched_cache[key] = build_schedule(self.kind, self.P, m, self.mesh.pp, forward_only=forward_only)
        return self._sched_cache[key]

    def train(self, mode: bool = True):
        self.training = mode
        for m in self.stages.values():
            m.train(mode)
        return self

    def eval(self):
        return self.train(False)

    @property
    def data_shards(self) -> int:
        """Number of disjoint per-step data shards (= samples per step / batch_size)."""
        return self.mesh.dp * (self.mesh.pp if self.kind == "rotate" else 1)

    def local_start(self, step_start: int, batch_size: int) -> int:
        """The ``start`` to pass to :meth:`run` for a step whose global batch begins at
        ``step_start`` (``batch_size`` samples per shard). ``rotate`` addresses its owners'
        shards itself, so it gets the start of its replica group's block."""
        if self.kind == "rotate":
            return step_start + self.mesh.dp_rank * self.mesh.pp * batch_size
        return step_start + self.mesh.dp_rank * batch_size

    def holds_first_stage(self) -> bool:
        return 0 in self.stages

    def holds_last_stage(self) -> bool:
        return (self.P - 1) in self.stages

    # ---------------------------------------------------------------------------------------
    def _boundary(self, producer_stage: int, mb: int):
        return self.spec.boundary_shape(producer_stage, mb), self.spec.boundary_dtype

    def _loss_scale(self, dataset, batch_size: int, global_batch: Optional[int]) -> float:
        """Per-sample (per-token for token models) loss weight: the summed gradients then equal
        d(mean loss over the global batch)/dθ, as ``nll_loss(reduction='mean')`` on one
        process (/root/reference/simple_distributed.py:111). Every schedule uses this."""
        gb = global_batch if global_batch is not None else batch_size * self.data_shards
        scale = 1.0 / float(gb)
        if self.spec.input_kind == "tokens":
            scale = scale / float(dataset.seq_len)
        return scale

    def _check_targets(self, dataset, start: int, n: int):
        """debug_sync: a label outside [0, classes) raises here. The fused heads (head_xent.hip,
        mlp_u8.hip) give such a row no loss term and no gradient, where torch's nll_loss in the
        reference (/root/reference/simple_distributed.py:111) raises."""
        spec = self.spec
        C = spec.vocab_size if spec.input_kind == "tokens" else spec.num_classes
        t = dataset.targets(start, n)
        lo, hi = int(t.min()), int(t.max())
        if lo < 0 or hi >= C:
            raise ValueError(f"target out of range [0, {C}) in samples [{start}, {start + n}): min {lo}, max {hi}")

    def run(self, dataset, start: int, batch_size: int, train: bool, global_batch: Optional[int] = None,
            step_optimizer: bool = True) -> StepResult:
        """One pipeline step over samples [start, start+batch_size) of ``dataset``.

        ``global_batch`` (default: batch_size * dp) sets the loss scale so that the summed
        gradients equal d(mean loss over the global batch)/dθ, matching a single-process
        ``nll_loss(..., reduction='mean')`` step on the whole batch.
        """
        t0 = time.perf_counter()
        dev = self.device
        rotate_a2a = self.kind == "rotate" and self.use_alltoall and self.P == 2
        if self.debug_sync and batch_size > 0:
            # rotate: heads run on rows of every owner of the replica group's block, not just this shard
            n_chk = batch_size * (self.mesh.pp if self.kind == "rotate" else 1)
            self._check_targets(dataset, start, n_chk)
        if batch_size <= 0:  # a DP replica with no samples in a ragged last batch
            if train:
                self.flat.zero_grad()
                self.grad_sync.reset()
                # still joins the collectives of its replica group, with the SAME collective sequence the
                # data-bearing ranks issue (rotate all-to-all: one all-reduce over the whole flat buffer, or the
                # two spans of the split weight gradient when the replicas run it: _planned_dp_spans)
                if rotate_a2a:
                    self._issue_planned_spans(self._planned_dp_spans())
                    join_side_streams()
                    self.grad_sync.finish_all()
                else:
                    join_side_streams()
                    self.grad_sync.finish()
                if step_optimizer:
                    join_side_streams()
                    self.optimizer.step()
                    self.global_step += 1
                self._advance_rng()
            z = torch.zeros(2, device=dev, dtype=torch.float32)
            return StepResult(z[0], z[1], 0, time.perf_counter() - t0)
        if train and step_optimizer and self._small_step_ok(batch_size):
            res = self._run_small_mlp_step(dataset, start, batch_size, global_batch, t0)
            if res is not None:
                return res
        if train and step_optimizer and self._cnn_step_ok(batch_size):
            return self._run_cnn_step(dataset, start, batch_size, global_batch, t0)
        if rotate_a2a:
            return self._run_rotate_alltoall(dataset, start, batch_size, train, global_batch, step_optimizer, t0)
        if self.kind == "rotate":
            # every rank owns a shard of ``batch_size`` samples at start + owner*batch_size,
            # cut into M/R micro-batches; the schedule sends them around the ring of peers
            R = self.mesh.pp
            per = split_sizes(batch_size, self.M // R)
            if len(per) * R != self.M:
                raise ValueError(f"rotate: batch {batch_size} too small for {self.M // R} micro-batches per rank")
            sizes, offs = [], []
            for owner in range(R):
                o = start + owner * batch_size
                for sz in per:
                    sizes.append(sz)
                    offs.append(o)
                    o += sz
        else:
            sizes = split_sizes(batch_size, self.M)
            offs = [start]
            for s in sizes[:-1]:
                offs.append(offs[-1] + s)
        M = len(sizes)
        sched = self.schedule(M, forward_only=not train)
        prog = sched.program(self.mesh.pp_rank)
        scale = self._loss_scale(dataset, batch_size, global_batch)
        # factored boundary gradient on a 2-stage neighbour pipeline whose ranks hold BOTH stages (Chimera's
        # mirror pipelines, the pp2dp placement): the head sends back its rank-C factor dl [mb, C] (40 B per row
        # for 784-128-10) instead of dx [mb, 128] (512 B), and the stage-0 rank rebuilds dx bit-identically with
        # its own replica of W2 (the mirror all-reduce keeps the replicas equal). Lossless: the same bytes of
        # information, 1024 -> 552 B per row over the pair's link.
        fact = (train and self.factored_boundary_grad and self.P == 2 and self.mesh.pp > 1 and 0 in self.stages
                and 1 in self.stages and getattr(self.stages[1], "supports_factored_grad", False))
        n_cls = self.stages[1].layers()[-1].out_features if fact else 0

        if train:
            self.flat.zero_grad()  # no-op when the previous optimizer step already cleared them
            self.flat.grads_zero = False
            self.grad_sync.reset()
        last_bwd = {}
        if train:
            for i, ins in enumerate(prog):
                if ins.op == OP_BWD:
                    last_bwd[ins.stage] = i

        ctxs: Dict[Tuple[int, int, int], dict] = {}
        local: Dict[Tuple[int, int, int, int], torch.Tensor] = {}
        outbox: Dict[Tuple[int, int, int, int], torch.Tensor] = {}
        inbox: Dict[Tuple[int, int, int, int], Tuple[object, torch.Tensor]] = {}
        stats = torch.zeros(2, device=dev, dtype=torch.float32)  # [loss_sum, correct]
        count = 0

        tm = PhaseTimer(dev, self.timing)

        def take(key, peer_rank_is_local: bool):
            if peer_rank_is_local:
                return local.pop(key)
            w, buf = inbox.pop(key)
            with tm.span("recv_wait", key[2]):
                w.wait()
            return buf

        for i, ins in enumerate(prog):
            op = ins.op
            if op == OP_RECV:
                mbsz = sizes[ins.mb]
                prod = ins.stage if ins.payload == PL_ACT else ins.stage - 1
                if fact and ins.payload == PL_GRAD:
                    shape, dt = (mbsz, n_cls), torch.float32
                else:
                    shape, dt = self._boundary(prod, mbsz)
                buf = self.bufs.get(("recv", ins.payload, ins.pipe, ins.stage, ins.mb), shape, dt)
                src = self.mesh.global_rank(self.mesh.dp_rank, ins.peer)
                w = self.transport.irecv(buf, src, message_tag(ins.payload, ins.pipe, ins.stage, ins.mb))
                inbox[(ins.payload, ins.pipe, ins.stage, ins.mb)] = (w, buf)
            elif op == OP_SEND:
                key = (ins.payload, ins.pipe, ins.stage, ins.mb)
                t = outbox.pop(key)
                dst = self.mesh.global_rank(self.mesh.dp_rank, ins.peer)
                self.transport.isend(t, dst, message_tag(*key))
            elif op == OP_FWD:
                mod = self.stages[ins.stage]
                mbsz, off = sizes[ins.mb], offs[ins.mb]
                if ins.stage == 0:
                    x = dataset.inputs(off, mbsz)
                    if x.device != dev:
                        x = x.to(dev, non_blocking=True)
                    if x.dtype == torch.uint8 and not mod.accepts_u8_pixels:
                        x = pixels_to_float(x)
                else:
                    prev_local = sched.task_rank(ins.mb, ins.stage - 1) == self.mesh.pp_rank
                    x = take((PL_ACT, ins.pipe, ins.stage - 1, ins.mb), prev_local)
                ctx = ctxs.setdefault((ins.pipe, ins.stage, ins.mb), {})
                if mod.is_last:
                    tgt = dataset.targets(off, mbsz)
                    if tgt.device != dev:
                        tgt = tgt.to(dev, non_blocking=True)
                    if fact:  # forward + loss + backward at once; dl waits in ctx for this micro-batch's OP_BWD
                        with tm.span("fwd", ins.stage):
                            ctx["dl"], n = mod.head_fwd_factored(x, tgt, scale, stats)
                        count += n
                    else:
                        with tm.span("fwd", ins.stage):
                            l, c, n = mod.head_fwd(x, tgt, ctx, train, scale, stats=stats)
                        if l is not None:  # stage did not accumulate in-kernel
                            stats[0] += l.float()
                            stats[1] += c.float()
                        count += n
                else:
                    with tm.span("fwd", ins.stage):
                        y = mod.fwd(x, ctx, train)
                    key = (PL_ACT, ins.pipe, ins.stage, ins.mb)
                    if sched.task_rank(ins.mb, ins.stage + 1) == self.mesh.pp_rank:
                        local[key] = y
                    else:
                        outbox[key] = y
                if not train:
                    ctxs.pop((ins.pipe, ins.stage, ins.mb), None)
            elif op == OP_BWD:
                mod = self.stages[ins.stage]
                ctx = ctxs.pop((ins.pipe, ins.stage, ins.mb))
                if mod.is_last:
                    if fact:
                        gx = ctx.pop("dl")
                    else:
                        with tm.span("bwd", ins.stage):
                            gx = mod.head_bwd(ctx)
                else:
                    nxt_local = sched.task_rank(ins.mb, ins.stage + 1) == self.mesh.pp_rank
                    gy = take((PL_GRAD, ins.pipe, ins.stage + 1, ins.mb), nxt_local)
                    with tm.span("bwd", ins.stage):
                        if fact:  # gy is the head's factor dl
                            s1 = self.stages[1]
                            gx = None
                            if not mod.bwd_from_factor(gy, s1.factor_weight(), ctx):
                                h = ctx["acts"][-1] if "acts" in ctx else ctx["y"]
                                gx = mod.bwd(s1.boundary_grad_from_factor(gy, h.detach()), ctx)
                        else:
                            gx = mod.bwd(gy, ctx)
                if ins.stage > 0:
                    key = (PL_GRAD, ins.pipe, ins.stage, ins.mb)
                    if sched.task_rank(ins.mb, ins.stage - 1) == self.mesh.pp_rank:
                        local[key] = gx
                    else:
                        outbox[key] = gx
                if last_bwd.get(ins.stage) == i:
                    join_side_streams()  # side-stream weight gradients (ops/linear.py SDML_WGRAD_STREAM) are done
                    self.grad_sync.stage_done(ins.stage)
            if self.debug_sync and dev.type == "cuda":
                torch.cuda.synchronize(dev)
        if outbox or inbox or local:
            raise RuntimeError(f"pipeline step left undelivered tensors: out={list(outbox)} "
                               f"in={list(inbox)} local={list(local)}")
        if self.transport is not None:
            with tm.span("send_drain"):
                self.transport.drain_sends()
        if train:
            with tm.span("grad_sync"):
                join_side_streams()
                self.grad_sync.finish()
            if step_optimizer:
                with tm.span("optim"):
                    join_side_streams()
                    self.optimizer.step()
                self.global_step += 1
            self._advance_rng()
        self.last_timing = tm.result()
        return StepResult(stats[0], stats[1], count, time.perf_counter() - t0)

    # ---------------------------------------------------------------------------------------
    def rotate_parts(self, waves: Sequence[int], R: int) -> List[List[List[int]]]:
        """``P[w][o][k]``: rows of owner ``o``'s wave ``w`` whose stage 1 runs on rank ``k``
        (``k == o``: the rows that stay on their owner). Every rank derives the same matrix, so all
        of them issue the same collectives. An owner's wave rows are laid out
        ``[local | to peer k1 | to peer k2 | ...]`` (peers ascending).

        ``cross_fraction`` None: classic rotate, an equal 1/R share per rank (the owner keeps the
        largest); else that fraction of every wave crosses to the peers (0: nothing crosses, pure
        data parallelism over replicated stages; parallel/placement.py chooses it from a link
        model)."""
        P = []
        phi = self.cross_fraction
        for b in waves:
            if R == 1:
                c = 0
            elif phi is None:
                c = b - split_sizes(b, R)[0]
            else:
                c = min(b, int(round(phi * b)))
            cs = split_sizes(c, R - 1) if c > 0 else []
            cs += [0] * (R - 1 - len(cs))
            rows = []
            for o in range(R):
                row = [0] * R
                row[o] = b - c
                for i, k in enumerate(k for k in range(R) if k != o):
                    row[k] = cs[i]
                rows.append(row)
            P.append(rows)
        return P

    def _run_rotate_alltoall(self, dataset, start, batch_size, train, global_batch, step_optimizer, t0):
        """``rotate`` for a 2-stage model, boundary as all-to-all (same math as the p2p form).

        Each rank owns ``batch_size`` samples at ``start + rank*batch_size``, cut into W =
        M/R waves. Per wave: stage 0 on the own chunk -> the rows assigned to peers
        (:meth:`rotate_parts`) are exchanged with ONE all-to-all on the transport's forward
        channel -> stage 1 (+ loss, + its backward) on the rows that stayed local and on the rows
        received -> their input-grads go back by the inverse all-to-all on the backward channel ->
        stage-0 backward over all own rows. The local rows never enter a collective (no self
        copy). Waves are issued so that wave w's exchange overlaps the compute of its neighbours;
        with RCCL the collectives run on their own streams and only the consumer kernels wait.

        Factored boundary gradient (stage 1 a single Linear + log_softmax, e.g. 784-128-10): the
        gradient stage 1 returns, (dl @ W) * (h > 0), has rank <= C per sample. Every rank holds
        W (stage weights are replicated here), so the head returns dl [n, C] and the OWNER
        rebuilds the gradient from its own copy of h -- bit-identical to the head's own dx
        (tests/test_kernels_gpu.py), and 40 instead of 512 bytes per sample on the return
        all-to-all. Stage 1's forward, loss, dW/db and optimizer step stay where they were.
        """
        mesh, dev = self.mesh, self.device
        R, me = mesh.pp, mesh.pp_rank
        s0, s1 = self.stages[0], self.stages[1]
        # factored boundary gradient: every rank holds stage 1's weights (they are replicated in
        # this placement), so the head sends back only its rank-C factor dl [n, C] and the owner
        # rebuilds d(loss)/dz0 = (dl @ W1) * (h > 0) from its own boundary activation h
        factored = (train and (R > 1 or self.factored_r1) and self.factored_boundary_grad
                    and getattr(s1, "supports_factored_grad", False))
        # every owner holds the same ``batch_size``, so every rank derives the same wave count
        # (fewer waves than M/R when the batch is smaller) and issues the same collectives
        waves = split_sizes(batch_size, max(1, self.M // R))
        W = len(waves)
        scale = self._loss_scale(dataset, batch_size, global_batch)
        # [loss_sum, correct]; a head that can overwrite it (supports_stats_init) initialises it on
        # its first call of the step, so no zero-fill is launched
        fresh = bool(getattr(s1, "supports_stats_init", False))
        stats = (torch.empty if fresh else torch.zeros)(2, device=dev, dtype=torch.float32)
        count = 0
        if train:
            self.flat.zero_grad()
            self.flat.grads_zero = False
            self.grad_sync.reset()
        woff = [0]
        for w in waves[:-1]:
            woff.append(woff[-1] + w)
        P = self.rotate_parts(waves, R)
        # rows crossing a link in wave w (all owners): 0 -> every rank skips that wave's collectives
        crossing = [sum(P[w][o][k] for o in range(R) for k in range(R) if k != o) for w in range(W)]

        def owner_part(o, w, k):  # (dataset start, size) of the rows of owner o's wave w that go to k
            row = P[w][o]
            off = 0 if k == o else row[o] + sum(row[j] for j in range(k) if j != o)
            return start + o * batch_size + woff[w] + off, row[k]

        tm = PhaseTimer(dev, self.timing)
        ctx0 = [dict() for _ in waves]
        hkeep = [None] * W  # factored: the owner's boundary activation per wave (ReLU mask source)
        hloc, recv, fwork = [None] * W, [None] * W, [None] * W
        # stage 0 expands the factor itself when it can (MLP first layer on uint8 pixels)
        fuse0 = factored and hasattr(s0, "bwd_from_factor") and hasattr(s1, "factor_weight")
        # nothing crosses GPUs: the head's gradient/stats reduction is deferred into stage 0's
        # weight-gradient reduction launch (one launch instead of two per wave); `pend[w]` must be
        # consumed or run
        defer = fuse0 and not any(crossing)
        pend = [None] * W
        if factored:
            gshape, gdt = (s1.layers()[-1].out_features,), torch.float32
        else:
            gshape, gdt = tuple(self._boundary(0, 1)[0][1:]), self.spec.boundary_dtype
        # both stages on this rank for the wave's local rows: ONE kernel runs stage 0's forward and
        # stage 1's forward + loss + backward (models/mlp.py fwd_head_fused; the boundary activation of
        # those rows never reaches HBM). SDML_FUSE_HEAD=0 runs them as separate kernels.
        fuse_fh = (train and fuse0 and self.fuse_head and hasattr(s0, "can_fuse_head"))
        gfused = [None] * W  # fused waves: the own-rows gradient buffer, local part written by the kernel
        for w, bw in enumerate(waves):  # stage 0 forward + scatter of the boundary activation
            x = dataset.inputs(start + me * batch_size + woff[w], bw)
            if x.device != dev:
                x = x.to(dev, non_blocking=True)
            if x.dtype == torch.uint8 and not s0.accepts_u8_pixels:
                x = pixels_to_float(x)
            L = P[w][me][me]
            if fuse_fh and L > 0 and self._can_fuse_head(s0, s1, x[:L]):
                # persistent per-wave buffers (stream-ordered reuse: this step's weight gradient consumes them before
                # the next step's forward rewrites them): no allocator / pool calls ahead of the step's first launch
                mask, G = self._fused_wave_bufs(w, bw, s0.layers()[0].out_features // 32, gshape, gdt)
                h = None
                if L < bw:  # the rows whose stage 1 runs on peers: plain forward, h is sent
                    with tm.span("fwd", 0):
                        h = s0.fwd(x[L:], {}, train, mask_out=mask[L:])
                tgt = dataset.targets(*owner_part(me, w, me))
                if tgt.device != dev:
                    tgt = tgt.to(dev, non_blocking=True)
                with tm.span("fwd", 1):
                    bound, pw = s0.fwd_head_fused(x[:L], s1, tgt, scale, stats, fresh, G[:L], mask[:L], None,
                                                  defer=defer)
                fresh = False
                count += L
                pend[w] = pw
                if bound is not None and L == bw:
                    G._sdml_amax = bound  # per-block bounds on |dl @ W2| (the weight gradient's dz scale)
                ctx0[w] = {"acts": [x.reshape(bw, -1)], "mask": mask}
                gfused[w] = G
                if crossing[w] == 0:
                    continue
                hx = h
            else:
                mask = None
                if fuse0 and x.dtype == torch.uint8 and s0.layers()[0].out_features % 32 == 0:
                    mask = torch.empty((bw, s0.layers()[0].out_features // 32), dtype=torch.int32, device=dev)
                with tm.span("fwd", 0):
                    h = s0.fwd(x, ctx0[w], train, mask_out=mask) if mask is not None else s0.fwd(x, ctx0[w], train)
                if factored:
                    hkeep[w] = h
                hloc[w] = h if L == bw else h[:L]
                if crossing[w] == 0:
                    continue
                hx = h[L:]
            in_splits = [0 if k == me else P[w][me][k] for k in range(R)]
            out_splits = [0 if o == me else P[w][o][me] for o in range(R)]
            buf = self.bufs.get(("a2a_fwd", w), (sum(out_splits),) + tuple(hx.shape[1:]), hx.dtype)
            fwork[w] = self.transport.all_to_all(buf, hx, out_splits, in_splits, channel="fwd")
            recv[w] = buf
        back, bwork = [None] * W, [None] * W
        # ... and when nothing else touches the gradients before the optimizer (one rank, no gradient
        # all-reduce, stepping this call), the last wave's reduction applies the optimizer step too
        fuse_step = (defer and train and step_optimizer and not self.grad_sync.enabled
                     and hasattr(self.optimizer, "fused_args") and hasattr(s0, "grad_span")
                     and hasattr(s1, "grad_span"))
        step_fused = [False]

        def run_pending(w):
            if pend[w] is not None:
                pend[w].run()
                pend[w] = None

        # the gradient all-reduce overlapped with the last wave's first-layer weight gradient (see __init__). The
        # decision depends only on rank-independent facts (model, placement, knob), so every replica issues the same
        # two spans; a rank whose batch the split kernels do not take issues them after its whole gradient
        dp_spans = self._planned_dp_spans() if (defer and train) else None

        spans_left = [dp_spans is not None]  # planned spans not issued yet (the split kernels did not run)

        def head(xin, tgt, w):  # stage 1 forward + loss (+ its backward) on one block of rows
            nonlocal fresh, count
            if tgt.device != dev:
                tgt = tgt.to(dev, non_blocking=True)
            if factored:
                with tm.span("fwd", 1):
                    if defer:
                        g, n, pend[w] = s1.head_fwd_factored(xin, tgt, scale, stats, stats_init=fresh,
                                                             defer_reduce=True)
                    else:
                        g, n = s1.head_fwd_factored(xin, tgt, scale, stats, stats_init=fresh)
                fresh = False
                count += n
                return g
            c1 = {}
            kw = {"stats_init": True} if fresh else {}
            with tm.span("fwd", 1):
                l, c, n = s1.head_fwd(xin, tgt, c1, train, scale, stats=stats, **kw)
            fresh = False
            if l is not None:
                stats[0] += l.float()
                stats[1] += c.float()
            count += n
            if not train:
                return None
            with tm.span("bwd", 1):
                return s1.head_bwd(c1)

        def stage0_bwd(w):
            if bwork[w] is not None:
                with tm.span("recv_wait", 1):
                    bwork[w].wait()
            gz = back[w]
            if factored and fuse0 and dp_spans is not None and w == W - 1:
                G, a1 = dp_spans
                ga = G // 2
                with tm.span("bwd", 0):
                    ok = s0.bwd_from_factor(gz, s1.factor_weight(), ctx0[w], head_pending=pend[w],
                                            groups=(0, ga, self.dp_split_blocks), final=False)
                    if ok:  # range 0 (and the head's reduction) done: its weight rows go on the links now
                        pend[w] = None
                        self.grad_sync.issue_span(0, a1)
                        s0.bwd_from_factor(gz, s1.factor_weight(), ctx0[w], groups=(ga, G - ga, self.dp_split_blocks))
                        # the rest: range 1's rows, every bias, the head (all written by now)
                        self.grad_sync.issue_span(a1, self.flat.grads.numel())
                        self.dp_split_steps += 1
                        spans_left[0] = False
                        hkeep[w] = back[w] = None
                        return
            if factored and fuse0:  # the factor goes straight into stage 0's weight-gradient kernel
                with tm.span("bwd", 0):
                    if pend[w] is not None:
                        sgd = None
                        if fuse_step and w == W - 1:
                            spans = [s0.grad_span(), s1.grad_span()]
                            if all(sp is not None for sp in spans):
                                sgd = self.optimizer.fused_args(spans)
                        done = s0.bwd_from_factor(gz, s1.factor_weight(), ctx0[w], head_pending=pend[w], sgd=sgd)
                        step_fused[0] = bool(done and sgd is not None and getattr(s0, "sgd_fused", False))
                    else:
                        done = s0.bwd_from_factor(gz, s1.factor_weight(), ctx0[w])
                if done:
                    pend[w] = None  # consumed (run inside the weight-gradient reduction)
                    hkeep[w] = back[w] = None
                    return
                run_pending(w)
            if factored:
                with tm.span("bwd", 1):
                    gz = s1.boundary_grad_from_factor(gz, hkeep[w])
                    hkeep[w] = None
            with tm.span("bwd", 0):  # every wave holds >= 1 owned row
                s0.bwd(gz, ctx0[w])
            back[w] = None

        # R > 1: wave w's stage-0 backward is issued right after its head, ahead of wave w+1's head:
        # the compute stream then has work while wave w+1's activations are still on the links
        # (the backward exchange runs on its own communicator and, factored, is small)
        interleave = train and R > 1
        for w, bw in enumerate(waves):  # stage 1 (+ loss + its backward): local rows, then received rows
            L = P[w][me][me]
            gloc = None
            if L > 0 and gfused[w] is None:  # (fused waves: the local rows' head already ran)
                gloc = head(hloc[w], dataset.targets(*owner_part(me, w, me)), w)
            hloc[w] = None
            if crossing[w] == 0:
                back[w] = gfused[w] if gfused[w] is not None else gloc
                if interleave:
                    stage0_bwd(w)
                continue
            if fwork[w] is not None:
                with tm.span("recv_wait", 0):
                    fwork[w].wait()
            srcs = [o for o in range(R) if o != me and P[w][o][me] > 0]
            grecv = None
            if srcs:
                tg = [dataset.targets(*owner_part(o, w, me)) for o in srcs]
                grecv = head(recv[w], tg[0] if len(tg) == 1 else torch.cat(tg), w)
            recv[w] = None
            if not train:
                continue
            # the received rows' gradients go back to their owners, into the own-rows gradient
            # buffer right after the local rows' part: [local | from peer k1 | from peer k2 ...]
            if grecv is None:  # nothing received this wave: still join the backward exchange
                grecv = torch.empty((0,) + gshape, dtype=gdt, device=dev)
            out_splits = [0 if k == me else P[w][me][k] for k in range(R)]
            in_splits = [0 if o == me else P[w][o][me] for o in range(R)]
            G = gfused[w]
            if G is None:
                G = self.bufs.get(("grad_own", w), (bw,) + gshape, gdt)
                if L > 0:
                    G[:L].copy_(gloc)
            bwork[w] = self.transport.all_to_all(G[L:], grecv, out_splits, in_splits, channel="bwd")
            back[w] = G
            if interleave:
                stage0_bwd(w)
        if train:
            if not interleave:
                for w in range(W):
                    stage0_bwd(w)
            for w in range(W):  # (nothing is left unless a stage-0 backward was skipped)
                run_pending(w)
            if spans_left[0]:  # the same two collectives as the replicas that ran the split
                self._issue_planned_spans(dp_spans)
            with tm.span("grad_sync"):  # both stages' gradients in one collective
                join_side_streams()
                self.grad_sync.finish_all()
            if step_optimizer:
                with tm.span("optim"):
                    if step_fused[0]:  # applied by the last weight-gradient reduction
                        self.optimizer.commit_fused()
                    else:
                        join_side_streams()
                        self.optimizer.step()
                self.global_step += 1
            self._advance_rng()
        if fresh:  # no head ran on this rank this step
            stats.zero_()
        self.last_timing = tm.result()
        return StepResult(stats[0], stats[1], count, time.perf_counter() - t0)

    def _can_fuse_head(self, s0, s1, x) -> bool:
        """s0.can_fuse_head(s1, x), memoised on what it depends on (stages, shape, strides, dtype, 16-B alignment)."""
        key = (id(s0), id(s1), tuple(x.shape), x.stride(), x.dtype, x.data_ptr() % 16, s0.plane_cache is not None)
        hit = self._fuse_ok.get(key)
        if hit is None:
            if len(self._fuse_ok) > 64:  # (a stream of odd shapes must not grow it without bound)
                self._fuse_ok.clear()
            hit = self._fuse_ok[key] = bool(s0.can_fuse_head(s1, x))
        return hit

    def _fused_wave_bufs(self, w, bw, nw, gshape, gdt):
        key = (w, bw, nw, tuple(gshape), gdt)
        hit = self._wave_bufs.get(key)
        if hit is None:
            if len(self._wave_bufs) > 16:  # (ragged batches: keep a bounded set; a dropped pair is freed by the allocator
                if self.graph_retain:  # once the stream no longer uses it - unless a captured graph may still write it)
                    self._wave_bufs_retired.extend(self._wave_bufs.values())
                self._wave_bufs.clear()
            mask = torch.empty((bw, nw), dtype=torch.int32, device=self.device)
            hit = self._wave_bufs[key] = (mask, self.bufs.get(("grad_own", w), (bw,) + tuple(gshape), gdt))
        return hit

    def _planned_dp_spans(self):
        """The split all-reduce spans every replica issues this step, or None. Only rank-independent facts decide
        (the knob, a gradient all-reduce, the rotate all-to-all form with nothing crossing GPUs, the model's first
        layer): a replica with no rows or a batch the split kernels do not take still issues the same spans."""
        if not (self.dp_split and self.grad_sync.enabled and self.kind == "rotate" and self.use_alltoall
                and self.P == 2 and 0 in self.stages and 1 in self.stages):
            return None
        R = self.mesh.pp
        if R > 1 and (self.cross_fraction is None or self.cross_fraction > 0):
            return None  # rows cross GPUs: one whole-buffer all-reduce (finish_all)
        if not (self.factored_boundary_grad and (R > 1 or self.factored_r1)
                and getattr(self.stages[1], "supports_factored_grad", False)
                and hasattr(self.stages[0], "bwd_from_factor") and hasattr(self.stages[1], "factor_weight")):
            return None
        return self._dp_split_spans(self.stages[0])

    def _issue_planned_spans(self, spans):
        if spans is not None:
            _, a1 = spans
            self.grad_sync.issue_span(0, a1)
            self.grad_sync.issue_span(a1, self.flat.grads.numel())

    def _dp_split_spans(self, s0):
        """(hidden groups G, end of range 0 in the flat gradient) when the first layer's weight gradient can
        run as two hidden-unit ranges with range 0's weight rows a prefix of the flat gradient buffer (then
        range 1's rows, the biases and the head's gradients form the contiguous rest), else None."""
        if not hasattr(s0, "hidden_groups"):
            return None
        G = s0.hidden_groups()
        if G < 2:
            return None
        lin = s0.layers()[0]
        g = lin.weight.grad
        if g is None or g.data_ptr() != self.flat.grads.data_ptr():
            return None
        return G, (G // 2) * 64 * lin.in_features

    # ---------------------------------------------------------------------------------------
    def _small_step_ok(self, batch_size: int) -> bool:
        """Both stages of the 784-128-10 MLP on this (only) rank, fp32 weights, a batch the one-launch
        step kernel takes, and no gradients pending from an earlier step_optimizer=False call."""
        if self._small_step is None:  # static: model shapes and placement only
            s = self.stages
            self._small_step = bool(
                self.device.type == "cuda" and self.mesh.world_size == 1 and self.P == 2 and 0 in s and 1 in s
                and self.optimizer.master is None and hasattr(s[0], "layers") and hasattr(s[1], "layers")
                and [tuple(l.weight.shape) for l in s[0].layers()] == [(128, 784)]
                and [tuple(l.weight.shape) for l in s[1].layers()] == [(10, 128)])
        # per call: timing / debug_sync may be switched on after the first step
        return (self._small_step and batch_size <= 128 and self.flat.grads_zero and not self.timing
                and not self.debug_sync and os.environ.get("SDML_SMALL_STEP", "1") != "0")

    def _run_small_mlp_step(self, dataset, start, batch_size, global_batch, t0):
        """The reference-size training step (B <= 128, e.g. its B = 60) in two kernel launches (ops.mlp_small_step):
        at this size the multi-kernel step is launch-bound."""
        dev = self.device
        x = dataset.inputs(start, batch_size)
        if x.device != dev:
            x = x.to(dev, non_blocking=True)
        x = x.reshape(batch_size, -1)
        if x.dtype not in (torch.float32, torch.uint8):
            x = x.float()
        tgt = dataset.targets(start, batch_size)
        if tgt.device != dev:
            tgt = tgt.to(dev, non_blocking=True)
        stats = torch.empty(2, device=dev, dtype=torch.float32)
        fc1, fc2 = self.stages[0].layers()[0], self.stages[1].layers()[0]
        if self._small_args is None:
            self._small_args = ops.mlp_small_step_args(fc1, fc2, self.optimizer)
        scale = self._loss_scale(dataset, batch_size, global_batch)
        if not ops.mlp_small_step(x.contiguous(), tgt.contiguous(), fc1, fc2, self.optimizer, scale, stats,
                                  self._small_args):
            return None
        self.optimizer.commit_fused(zero_grad=True, planes_current=False)
        self.global_step += 1
        self._advance_rng()
        self.last_timing = {}
        self.fast_steps["mlp_small"] += 1
        return StepResult(stats[0], stats[1], batch_size, time.perf_counter() - t0)

    def _cnn_step_ok(self, batch_size: int) -> bool:
        """Both stages of the reference CNN on this (only) rank, training mode, fp32 weights, no gradients
        pending from an earlier step_optimizer=False call: the two-launch step (ops.ref_cnn_step)."""
        if self._cnn_step is None:
            from ..models.ref_cnn import Network1Stage, Network2Stage

            s = self.stages
            self._cnn_step = bool(
                self.device.type == "cuda" and self.mesh.world_size == 1 and self.P == 2 and 0 in s and 1 in s
                and isinstance(s[0], Network1Stage) and isinstance(s[1], Network2Stage)
                and self.optimizer.master is None)
        # M == 1 only: the per-stage path draws one host dropout seed per micro-batch and stage, the
        # two-launch step draws two per step, so only at M == 1 do both paths draw the same masks
        return (self._cnn_step and self.M == 1 and 0 < batch_size <= 4096 and self.flat.grads_zero
                and self.training and self.stages[0].training and self.stages[1].training and not self.timing
                and not self.debug_sync and os.environ.get("SDML_SMALL_STEP", "1") != "0")

    def _run_cnn_step(self, dataset, start, batch_size, global_batch, t0):
        """The reference's own workload (its CNN at B = 60) as ONE per-sample kernel (stage 0 forward, stage 1
        forward + NLL + backward, stage 0 backward) + ONE reduction/SGD kernel: the three-kernel step with
        per-block weight-gradient atomics, a separate SGD launch and a dropout-counter launch was launch- and
        atomic-bound (profiles/r3_ref_cnn_kernel_stats.txt). Dropout seeds are drawn in the same order as the
        per-stage path (stage 0, then stage 1), so at M = 1 (the only case _cnn_step_ok admits) both draw the
        same masks."""
        from ..models.ref_cnn import _draw_seed

        dev = self.device
        x = dataset.inputs(start, batch_size)
        if x.device != dev:
            x = x.to(dev, non_blocking=True)
        x = pixels_to_float(x)
        if x.dtype != torch.float32:
            x = x.float()
        tgt = dataset.targets(start, batch_size)
        if tgt.device != dev:
            tgt = tgt.to(dev, non_blocking=True)
        s0, s1 = self.stages[0], self.stages[1]
        seed0 = _draw_seed() if s0.conv2_drop.p > 0 else 0
        seed1 = _draw_seed() if s1.p > 0 else 0
        stats = torch.empty(2, device=dev, dtype=torch.float32)
        scale = self._loss_scale(dataset, batch_size, global_batch)
        if self._cnn_args is None:
            self._cnn_args = ops.ref_cnn_step_args(s0, s1, self.optimizer)
        ops.ref_cnn_step(x.contiguous(), tgt.contiguous(), s0, s1, self.optimizer, scale, stats,
                         self.step_ctr if self._uses_rng else None, seed0, seed1, self._cnn_args)
        self.optimizer.commit_fused(zero_grad=True, planes_current=False)
        self.global_step += 1  # (the kernel advanced the device dropout counter)
        self.last_timing = {}
        self.fast_steps["cnn"] += 1
        return StepResult(stats[0], stats[1], batch_size, time.perf_counter() - t0)

    def reduce_metrics(self, res: StepResult, group=None) -> Tuple[float, int, int]:
        """Sum (loss, correct, count) over all last-stage holders (world). Host-syncs."""
        v = torch.stack([res.loss_sum.double(), res.correct.double(),
                         torch.tensor(float(res.count), dtype=torch.float64).to(res.loss_sum.device)])
        if self.mesh.tp_rank != 0:  # a tensor-parallel stage computes the loss on every tp rank
            v.zero_()
        if self.mesh.world_size > 1:
            # every pipeline's last stage contributes once; the other ranks contribute zeros
            self.transport.all_reduce(v, group=group, async_op=False)
        v = v.cpu()
        return float(v[0]), int(v[1]), int(v[2])

    def state_dicts(self) -> Dict[int, dict]:
        return {s: {k: v.detach().cpu().clone() for k, v in m.state_dict().items()} for s, m in self.stages.items()}

    def parameters_vector(self) -> torch.Tensor:
        return self.flat.params.detach().clone()
